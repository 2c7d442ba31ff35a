# occupancy sweep of the headline config (dev)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for o in ${OCCS:-0.35 0.7 1.0 1.5 2.5}; do
  timeout -k 10 200 python tools/quick_time.py 512 5000000 ${K:-8} $o > gpurun_out/sweep_$o.log 2>&1 || { cat gpurun_out/sweep_$o.log; exit 1; }
  tail -1 gpurun_out/sweep_$o.log
done
