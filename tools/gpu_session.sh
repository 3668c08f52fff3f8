# One GPU call, several named steps; every step is time-limited and the session stops at the
# first failure (no retries).  Usage: bash tools/gpu_session.sh STEP [STEP ...]
#   tests          pytest -m gpu                           -> gpurun_out/gpu_tests.log
#   smoke          __graft_entry__.smoke()                 -> gpurun_out/smoke.log
#   bench          the default `python bench.py` line      -> gpurun_out/bench.json
#   bench20        bench.py --steps 20 --warmup 3 --also-philox --no-cpu-baseline
#   bench50        bench.py --steps 50 --warmup 5 --also-philox --no-cpu-baseline
#   map            tools/mapbench.py                       -> gpurun_out/mapbench.json
#   c5             tools/c5bench.py --scans 4096 --reps 2  -> gpurun_out/c5.json
#   issue          tools/ubench_issue (built in-tree)      -> gpurun_out/ubench_issue.json
#   profile:TAG    tools/profile_session.sh TAG (kernel trace + PMC passes)
#   ab             tools/ab_multi.sh over $LIBS (C3 A/B of library builds, $REPS rounds)
#   ksweep         tools/ksweep.sh (per-step time vs timed steps)
#   chunkphase     tools/chunkphase.sh (chunk_kernel instructions per phase; variants built beforehand)
#   rehearse2      the driver's N > 1 launch (torch.distributed.run, 2 ranks, --no-c4) with every rank
#                  on device 0 (LSLAM_RANK_DEVICE=0)      -> gpurun_out/rehearsal_2ranks.log
#   c4one          bench.py --gpus 1 --c4: the whole 65,536-scan C4 leg at one rank -> gpurun_out/c4one.json
#   rehearse2c4    as rehearse2 with the C4 leg ON over RCCL (expected: RCCL refuses two ranks on one
#                  device, reported as the leg's {"error"}, main line intact) -> gpurun_out/rehearsal_2ranks_c4.log
#   rehearse2host  as rehearse2c4 with --c4-transport host (the gather through host TCP, so shared
#                  memory, pinning, H2D, pipeline, gather plan and D2H run in two processes)
#                                                          -> gpurun_out/rehearsal_2ranks_host.log
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}; mkdir -p gpurun_out
fail() { echo "step $1 failed"; tail -30 "$2"; exit 1; }
for step in "$@"; do
  echo "== $step"
  case $step in
    tests)
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || fail $step gpurun_out/gpu_tests.log
      tail -1 gpurun_out/gpu_tests.log ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || fail $step gpurun_out/smoke.log
      tail -1 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || fail $step gpurun_out/bench.err
      tail -1 gpurun_out/bench.json ;;
    bench20|bench50)
      k=${step#bench}; w=$([ $k = 20 ] && echo 3 || echo 5)
      timeout -k 10 300 python -u bench.py --steps $k --warmup $w --also-philox --no-cpu-baseline > gpurun_out/$step.json 2> gpurun_out/$step.err || fail $step gpurun_out/$step.err
      python3 -c "import json; d=json.load(open('gpurun_out/$step.json')); r=d['roofline']; print('C3', d['value'], d['ms_per_step'], 'rng', r['kernel_ms'], 'frac', r['frac'], 'consensus', r.get('consensus', {}).get('ms'), 'philox', d.get('philox_scans_per_s'))" ;;
    map)
      timeout -k 10 300 python -u tools/mapbench.py > gpurun_out/mapbench.json 2> gpurun_out/mapbench.err || fail $step gpurun_out/mapbench.err
      cat gpurun_out/mapbench.json ;;
    c5)
      timeout -k 10 300 python -u tools/c5bench.py --scans 4096 --reps 2 > gpurun_out/c5.json 2> gpurun_out/c5.err || fail $step gpurun_out/c5.err
      cat gpurun_out/c5.json ;;
    issue)
      timeout -k 10 60 tools/ubench_issue > gpurun_out/ubench_issue.json 2>&1 || fail $step gpurun_out/ubench_issue.json
      cat gpurun_out/ubench_issue.json ;;
    profile:*)
      bash tools/profile_session.sh ${step#profile:} || exit 1 ;;
    ab)
      bash tools/ab_multi.sh || exit 1 ;;
    ksweep)
      bash tools/ksweep.sh || exit 1 ;;
    chunkphase)
      bash tools/chunkphase.sh || exit 1 ;;
    rehearse2)
      LSLAM_RANK_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --no-c4 --steps 20 --warmup 3 \
        > gpurun_out/rehearsal_2ranks.log 2>&1 || fail $step gpurun_out/rehearsal_2ranks.log
      tail -1 gpurun_out/rehearsal_2ranks.log ;;
    c4one)
      timeout -k 10 400 python -u bench.py --gpus 1 --c4 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/c4one.json 2> gpurun_out/c4one.err || fail $step gpurun_out/c4one.err
      python3 -c "import json; d=json.load(open('gpurun_out/c4one.json')); print('C3', d['value'], d['ms_per_step'], 'coupled', d.get('coupled'), 'c4', d.get('c4'))" ;;
    rehearse2c4|rehearse2host)
      tr=$([ $step = rehearse2host ] && echo host || echo rccl)
      LSLAM_RANK_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --c4 --c4-transport $tr --c4-timeout 120 \
        --steps 20 --warmup 3 > gpurun_out/rehearsal_2ranks_$tr.log 2>&1 || fail $step gpurun_out/rehearsal_2ranks_$tr.log
      tail -1 gpurun_out/rehearsal_2ranks_$tr.log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
