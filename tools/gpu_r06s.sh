set -o pipefail
bash tools/gpu_envab.sh r06s_share abr6/libptv_dev6.so "--share 2/8 --steps 20 --warmup 3" "PTV_BIN_SORT=0; -" &&
bash tools/gpu_envab.sh r06s_filter abr6/libptv_dev6.so "--method filter --steps 10 --warmup 3" "PTV_BIN_SORT=0; -" &&
bash tools/gpu_envab.sh r06s_near abr6/libptv_dev6.so "--method nearest --steps 10 --warmup 3" "PTV_BIN_SORT=0; -"
