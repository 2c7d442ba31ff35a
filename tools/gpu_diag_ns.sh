set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/diag_ns.py 2e307 && PTV_LIB=$(realpath ab/libptv_nsst.so) PTV_RBF_NS=0 timeout -k 10 200 python tools/diag_ns.py 2e307 && timeout -k 10 200 python tools/diag_ns.py 1.0
