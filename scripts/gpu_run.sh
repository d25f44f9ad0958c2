#!/bin/bash
# One runner for every GPU-box recipe (replaces the per-experiment gpu_*.sh of rounds 1-2).
# Usage: scripts/gpu_run.sh TAG STEP [STEP ...]; output under gpurun_out/TAG. Steps run in order,
# each under its own time limit; the first failing step ends the run (set -e).
#   tests[:PATTERN]      pytest -m gpu (optionally -k PATTERN), verbose log
#   smoke                __graft_entry__.smoke()
#   bench:CFG[:ARGS]     bench.py --config CFG (ARGS: extra bench args, comma-separated) -> bench_CFG.json
#   default              bench.py with no arguments (the driver's N = 1 line) -> bench_default.json
#   prof:CFG             rocprofv3 kernel trace/stats + FETCH_SIZE / WRITE_SIZE passes (profile_traffic.sh)
#   td:CFG               TD roof PMC pass of the bench step and the td_gather peak (pmc_td_roof.sh)
#   pmc:CFG              the TD / TCP / SQ counter groups (pmc_td.sh)
#   ab:ROUNDS:SPP:SCENES A/B of build_variants/*.so (ab_variants.py), SCENES comma-separated
#   rehearse:N           bench.py under torchrun with N ranks all on device 0 over gloo (the driver's launch)
#   inflight             scripts/frames_in_flight.py: one context vs two frames in flight on two streams
#   subpk:SCENE          scripts/shadow_packets.py under rocprofv3: per-lane vs 16-lane sub-packet any-hit kernels
#   vparity              scripts/variant_parity.py: every build_variants/*.so bit-exact vs the oracle
#   overlap              scripts/overlap_probe.py: exchange kernels / copies beside the persistent trace
#   diag:CFG             one MFX_DIAG_ITER=1 frame (per-iteration ray counts and stage times)
#   dispatch:CFG[:SPP]   per-dispatch duration and HBM bytes of one frame (kernel trace + FETCH_SIZE and
#                        WRITE_SIZE passes, scripts/per_dispatch.py) -> dispatch_CFG.txt
#   diagab:SCENE:SPP     per-iteration stage times of every build_variants/*.so (with its .env), 2 rounds
#   iterstats:SCENE:SPP  per-bounce node / leaf / primitive visits per ray (scripts/iter_stats.py)
#   sharetrace:PARTS:NIF rocprofv3 kernel trace of one rank's 1/PARTS share over NIF contexts (comma list)
#                        (scripts/share_trace.py) and its timeline (scripts/share_timeline.py)
#   latroofvar:NAME:SCENE[:SPP]  latency roof of build_ab/NAME.so with its stamp builds NAME_st1/_st2
#   tdvar:NAME:CFG       TD roof of build_ab/NAME.so
#   vparityab            scripts/variant_parity.py on every build_ab/*.so
#   churn                trace time of contexts created after others were destroyed
#   sampletime           mfx_sample's host timeline per band, bench state vs a lone process
#   sampletrace          mfx_sample under rocprofv3 kernel + memory-copy trace (scripts/sample_trace.py)
#   sharequeues:K        K strong-share children under a kernel trace: HW queue ids per rank (share_queues.py)
#   py:SCRIPT[:ARGS]     scripts/SCRIPT.py ARGS (comma-separated) -> SCRIPT.json
#   latroof:SCENE:SPP    latency roof of k_extend / k_shadow from the stamp builds build_variants/st1.so,
#                        st2.so (scripts/latency_roof.py) -> latency_SCENE.json
set -e
# the hardware queues bench.py would relaunch itself with (so rocprofv3 sees one process)
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
for step in "$@"; do
  IFS=: read -r kind a1 a2 a3 <<< "$step"
  echo "== $step $(date +%T)" | tee -a $O/steps.log
  case $kind in
    tests)
      K=(); [ -n "$a1" ] && K=(-k "$a1")
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${K[@]}" \
        > $O/pytest_gpu.log 2>&1
      tail -1 $O/pytest_gpu.log ;;
    smoke)
      timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      cat $O/smoke.log ;;
    bench)
      X=(); [ -n "$a2" ] && IFS=, read -ra X <<< "$a2"
      timeout -k 10 420 python3 bench.py --config $a1 "${X[@]}" > $O/bench_$a1.json 2> $O/bench_$a1.err
      python3 -c "import json; d=json.load(open('$O/bench_$a1.json')); print('$a1', d['value'], d['ms_per_step'])" ;;
    default)
      timeout -k 10 420 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
      python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['value'], d['ms_per_step'])" ;;
    prof)
      bash scripts/profile_traffic.sh ${TAG}_$(echo $a1 | tr A-Z a-z) --config $a1 > $O/prof_$a1.log 2>&1 ;;
    td)
      make -s -C scripts/ubench td_gather sload > /dev/null 2>&1 || true
      bash scripts/pmc_td_roof.sh ${TAG}_$(echo $a1 | tr A-Z a-z) --config $a1 > $O/td_$a1.log 2>&1 ;;
    pmc)
      bash scripts/pmc_td.sh ${TAG}_$(echo $a1 | tr A-Z a-z) --config $a1 > $O/pmc_$a1.log 2>&1 ;;
    ab)
      IFS=, read -ra SC <<< "$a3"
      for sc in "${SC[@]}"; do
        echo "== $sc" >> $O/ab.txt
        MFX_AB_DIR=${MFX_AB_DIR:-build_ab} timeout -k 10 900 python3 scripts/ab_variants.py scenes/$sc $a1 $a2 >> $O/ab.txt 2>&1
      done
      grep -E "==|SUMMARY" $O/ab.txt ;;
    rehearse)
      # the driver's N-rank launch on this one GPU: every rank on device 0, gloo (RCCL refuses two
      # ranks on one device); a rehearsal of the code path, not a scaling figure
      MFX_BENCH_DEVICE=0 MFX_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 \
        --nproc-per-node=$a1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $a1 --no-cpu-baseline \
        --no-stats --steps 5 --warmup 1 > $O/rehearse_$a1.json 2> $O/rehearse_$a1.err
      python3 -c "import json; d=json.load(open('$O/rehearse_$a1.json')); print('rehearse', d['n_gpus'], d['scaling'], d['value'], d['config']['global_spp_per_step'], d['config']['frames_in_flight'])" ;;
    inflight)
      timeout -k 10 300 python3 scripts/frames_in_flight.py --modes 1,2,3 > $O/inflight.json 2> $O/inflight.err
      cat $O/inflight.json ;;
    subpk)
      D=$R/$O/subpk_$a1
      mkdir -p $D
      (cd /tmp && export TMPDIR=/tmp &&
       timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- \
         python3 $R/scripts/shadow_packets.py --scene $R/scenes/$a1 > $D/run.json 2> $D/run.err)
      cat $D/run.json
      grep -h "anyhit" $D/trace/*kernel_stats.csv | cut -d, -f1-4 ;;
    vparity)
      timeout -k 10 600 python3 scripts/variant_parity.py build_variants/*.so > $O/vparity.txt 2>&1
      cat $O/vparity.txt ;;
    overlap)
      timeout -k 10 300 python3 scripts/overlap_probe.py > $O/overlap.json 2> $O/overlap.err
      cat $O/overlap.json ;;
    diag)
      MFX_DIAG_ITER=1 timeout -k 10 300 python3 bench.py --config $a1 --steps 1 --warmup 1 --no-cpu-baseline \
        --no-render-api --no-stats > $O/diag_$a1.json 2> $O/diag_$a1.txt ;;
    dispatch)
      D=$R/$O/dispatch_$a1
      B="$R/bench.py --config $a1 --steps 1 --warmup 1 --no-cpu-baseline --no-stats --no-render-api"
      [ -n "$a2" ] && B="$B --spp $a2" && D=${D}_$a2
      mkdir -p $D
      (cd /tmp && export TMPDIR=/tmp &&
       timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- python3 $B > $D/trace.log 2>&1 &&
       timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 $B > $D/fetch.log 2>&1 &&
       timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 $B > $D/write.log 2>&1)
      python3 scripts/per_dispatch.py $D | tee $O/$(basename $D).txt ;;
    diagab)
      for round in 0 1; do
        for l in build_variants/*.so; do
          E=(); [ -f ${l%.so}.env ] && E=($(cat ${l%.so}.env))
          env "${E[@]}" timeout -k 10 120 python3 scripts/diag_variant.py $l scenes/$a1 $a2 >> $O/diagab.txt 2>&1
        done
      done
      grep -E "^---|gen 0 iter" $O/diagab.txt | grep -v "trace 0" | grep -A4 -E "^---" > $O/diagab_summary.txt || true
      cat $O/diagab_summary.txt ;;
    iterstats)
      timeout -k 10 300 python3 scripts/iter_stats.py scenes/$a1 $a2 | tee $O/iterstats_$a1.txt ;;
    sharetrace)
      D=$R/$O/sharetrace_${a1}_$(echo $a2 | tr , _)
      mkdir -p $D
      (cd /tmp && export TMPDIR=/tmp &&
       timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- \
         python3 $R/scripts/share_trace.py --parts $a1 --nif $a2 --steps 20 > $D/run.json 2> $D/run.err)
      cat $D/run.json
      python3 scripts/share_timeline.py $D/trace | tee $D/timeline.txt ;;
    latroof)
      timeout -k 10 900 python3 scripts/latency_roof.py --scene scenes/$a1 --spp ${a2:-64} \
        --out $O/latency_$(basename $a1 .xml).json > $O/latroof.log 2>&1
      tail -5 $O/latroof.log ;;
    latroofvar)
      # a variant's latency roof: build_ab/NAME.so with its stamp builds build_ab_st/NAME_st1.so, _st2.so
      timeout -k 10 900 python3 scripts/latency_roof.py --scene scenes/$a2 --spp ${a3:-64} --lib build_ab/$a1.so \
        --st1 build_ab_st/${a1}_st1.so --st2 build_ab_st/${a1}_st2.so --st3 none \
        --out $O/latency_${a1}_$(basename $a2 .xml).json > $O/latroof_$a1.log 2>&1
      tail -5 $O/latroof_$a1.log ;;
    tdvar)
      # the TD roof of build_ab/NAME.so (MFX_LIB_PATH) on config CFG
      make -s -C scripts/ubench td_gather sload > /dev/null 2>&1 || true
      MFX_LIB_PATH=$R/build_ab/$a1.so bash scripts/pmc_td_roof.sh ${TAG}_${a1}_$(echo $a2 | tr A-Z a-z) --config $a2 \
        > $O/td_${a1}_$a2.log 2>&1 ;;
    vparityab)
      timeout -k 10 600 python3 scripts/variant_parity.py build_ab/*.so > $O/vparityab.txt 2>&1
      cat $O/vparityab.txt ;;
    churn)
      # a context's trace time after others came and went (scripts/context_churn_probe.py)
      timeout -k 10 600 python3 scripts/context_churn_probe.py > $O/churn.json 2> $O/churn.err
      cat $O/churn.json ;;
    sampletime)
      # mfx_sample's host timeline (MFX_SAMPLE_TIMING=1: each band's arrival and copy) in bench.py's
      # process state and in a process that only samples (scripts/sample_in_bench_probe.py)
      SAMPLE_PROBE_SETTINGS=${SAMPLE_PROBE_SETTINGS:-bands4_streams1,unbanded} MFX_SAMPLE_TIMING=1 timeout -k 10 300 \
        python3 scripts/sample_in_bench_probe.py > $O/sampletime_bench.json 2> $O/sampletime_bench.err
      SAMPLE_PROBE_SETTINGS=${SAMPLE_PROBE_SETTINGS:-bands4_streams1,unbanded} MFX_SAMPLE_TIMING=1 timeout -k 10 300 \
        python3 scripts/sample_in_bench_probe.py --lone > $O/sampletime_lone.json 2> $O/sampletime_lone.err
      (lscpu | grep -i numa; grep Cpus_allowed_list /proc/self/status) > $O/sampletime_numa.txt || true
      cat $O/sampletime_bench.json $O/sampletime_lone.json $O/sampletime_numa.txt ;;
    sampletrace)
      # mfx_sample under a kernel + memory-copy trace, banded vs unbanded (scripts/sample_trace.py)
      D=$R/$O/sampletrace
      mkdir -p $D
      (cd /tmp && export TMPDIR=/tmp &&
       timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/trace -o run -- \
         python3 $R/scripts/sample_trace.py > $D/run.json 2> $D/run.err)
      cat $D/run.json
      python3 scripts/sample_trace.py --timeline $D/trace > $D/timeline.txt; tail -40 $D/timeline.txt ;;
    sharequeues)
      # the strong-share child under a kernel trace, a1 times: which HW queues its contexts used
      for i in $(seq 1 $a1); do
        D=$R/$O/sharequeues/p$i
        mkdir -p $D
        (cd /tmp && export TMPDIR=/tmp &&
         timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run -- \
           python3 $R/bench.py --steps 20 --strong-share-child 0 0 > $D/run.json 2> $D/run.err)
      done
      python3 scripts/share_queues.py $O/sharequeues | tee $O/sharequeues.txt ;;
    py)
      # py:SCRIPT[:ARGS] -- scripts/SCRIPT.py with comma-separated ARGS -> SCRIPT.json / SCRIPT.err
      X=(); [ -n "$a2" ] && IFS=, read -ra X <<< "$a2"
      timeout -k 10 300 python3 scripts/$a1.py "${X[@]}" > $O/$a1.json 2> $O/$a1.err
      tail -3 $O/$a1.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
