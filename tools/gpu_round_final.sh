#!/bin/bash
# Round-end evidence on HEAD in one GPU call: the whole -m gpu suite + smoke(), the rocprofv3
# kernel-trace stats and the FETCH_SIZE / WRITE_SIZE passes of the default bench command (turned
# into profiles/traffic_<tag>.json on the box, so that every bench line after it carries the
# measured traffic of this very build), then every bench line (tools/gpu_lines.sh).
# usage: gpurun -- bash tools/gpu_round_final.sh r05
set -o pipefail
tag=${1:-r05}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA -s --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${tag}_tests.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${tag}_tests.log | head -20; exit $rc; fi
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -5 gpurun_out/${tag}_smoke.log; exit 1; }
  tail -1 gpurun_out/${tag}_smoke.log
fi
bash tools/collect_profiles.sh ${tag} || exit 1
tail -4 profiles/${tag}_summary.txt
# profiles/ on the box is not merged back: copy what collect_profiles wrote
mkdir -p gpurun_out/profiles_box
cp profiles/traffic_${tag}.json profiles/${tag}_summary.txt profiles/${tag}_kernel_stats.csv gpurun_out/profiles_box/
[ -n "$SKIP_LINES" ] || bash tools/gpu_lines.sh ${tag}
