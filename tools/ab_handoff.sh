cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for v in "AICP_SEQ_HOST_HANDOFF=0" "AICP_SEQ_HOST_HANDOFF=1" "AICP_SEQ_HOST_HANDOFF=0 AICP_R2_PRIO_LO=1" "AICP_SEQ_HOST_HANDOFF=1 AICP_R2_PRIO_LO=1"; do
    env $v AICP_PROF=1 timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-batched > gpurun_out/ab.log 2>&1 || exit 1
    echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab.log | head -1)"; grep "device ms" gpurun_out/ab.log | tail -1
  done
done
