# The one GPU runner (run under gpurun): a sequence of named steps, each with its own time limit;
# the first failure ends the script (no retries).  Outputs under gpurun_out/$ROUND/.
#   STEPS="smoke tests fullparity bench prof" ROUND=r05 bash tools/gpu_round.sh
# smoke      __graft_entry__.smoke()
# tests      pytest -m gpu (every parity test; PYTEST_K="expr" narrows it, PYTEST_FILES the files)
# abtests    pytest tools/ab_tests (the A/B library tools/ab/libkdstep_ab.so: build it locally with
#            csrc/build.py --ab before the call; it travels with the tree)
# fullparity c1 at full depth vs the fp32 oracle + the plain-bf16 floor + the teacher-stream A/B
#            (tools/parity_report.py --full-depth) -> full_depth.json
# fp8parity  c1 at full depth with the fp8 (e4m3, lm_mlp) teacher of c4 vs the same fp32 oracle
#            -> full_depth_fp8.json
# kindparity every other module (DT phases 1-3, FB, BD) at full depth vs the fp32 oracle
#            (FULL_KINDS, default "dt1 dt2 dt3 fb bd") -> full_depth_kinds.json
# sunparity  c1 at full depth on the SUNRGBD 480x640 geometry (5 tiles, L 2980) vs the fp32 oracle -> full_depth_sunrgbd.json
# sunbench   bench.py --image 480x640 (the c1 line at SUNRGBD geometry) -> bench_c1_sunrgbd.json
# c4parity   BASELINE c4 itself at full depth (DT phase 3 + fp8 lm_mlp teacher) vs the fp32 oracle -> c4_full_depth.json
# hnprofile  the student's hidden-state error vs the fp32 oracle at SigLIP / Qwen2 depths -> depth_profile.json
# fp8study   tools/fp8_c4_study.py: the c4 KD term's fp8-vs-bf16 move split into LoCa top-2 flips and smooth change,
#            product library, then the A/B library with the GEMM k-loop stagger off -> fp8_c4*.json
# parity     the reduced-depth fixtures' per-term / per-parameter report -> parity.json
# ntx        tools/ntx_bias_study.py (NT-Xent-only bias gradients) -> ntx_bias.json
# bench      bench.py (the driver's default line; BENCH_ARGS appended) -> bench.json
# c2|c3|c4   bench.py --config cN --no-cpu-baseline -> bench_cN.json
# ab         the c1 bench once per setting in AB_SETS ("|"-separated env settings, read by the A/B
#            library only when KDSTEP_LIB points at it; bench flags in AB_ARGS) -> ab_<i>.json
# prof       rocprofv3 --kernel-trace --stats of a serialized bench -> prof/ (kernel_stats.csv)
# step       kernel trace of the concurrent bench -> step_breakdown.txt
# pmc        HBM traffic per kernel (tools/pmc_bench.sh: FETCH / WRITE passes)
# pmcstep    MFMA-busy / wave cycles / clock per kernel family (tools/pmc_bench.sh mfma; wall times from
#            the prof step's kernel trace, so list prof first) -> pmc_step.json
# blas       PMC clock / MFMA-busy / FETCH of kd_gemm vs hipBLASLt on the big shapes (tools/pmc_vs_blas.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ROUND=${ROUND:-r06}
O=gpurun_out/$ROUND
mkdir -p $O
STEPS=${STEPS:-"tests parity bench prof"}
BENCH_ARGS=${BENCH_ARGS:-""}
fail() { echo "$1 failed"; tail -${3:-30} "$2"; exit 1; }
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    smoke)  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
            tail -1 $O/smoke.log ;;
    tests)  timeout -k 10 1100 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q --timeout 900 --timeout-method thread \
                -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1 || fail pytest $O/pytest_gpu.log 60
            tail -2 $O/pytest_gpu.log ;;
    abtests) timeout -k 10 600 python -u -m pytest tools/ab_tests -m gpu -x -q --timeout 300 --timeout-method thread \
                -p no:cacheprovider > $O/pytest_ab.log 2>&1 || fail abtests $O/pytest_ab.log 40
            tail -2 $O/pytest_ab.log ;;
    fp8parity) timeout -k 10 900 python -u tools/parity_report.py --full-depth --teacher-fp8 lm_mlp \
                --out $O/full_depth_fp8.json > $O/full_depth_fp8.log 2>&1 || fail fp8parity $O/full_depth_fp8.log ;;
    kindparity) timeout -k 10 1100 python -u tools/parity_report.py --full-depth-kinds ${FULL_KINDS:-dt1 dt2 dt3 fb bd} \
                --out $O/full_depth_kinds.json > $O/full_depth_kinds.log 2>&1 || fail kindparity $O/full_depth_kinds.log ;;
    fullparity) timeout -k 10 900 python -u tools/parity_report.py --full-depth --floor --teacher-stream-ab \
                --out $O/full_depth.json > $O/full_depth.log 2>&1 || fail fullparity $O/full_depth.log ;;
    sunparity) timeout -k 10 900 python -u tools/parity_report.py --full-depth --image 480x640 \
                --out $O/full_depth_sunrgbd.json > $O/full_depth_sunrgbd.log 2>&1 || fail sunparity $O/full_depth_sunrgbd.log ;;
    sunbench) timeout -k 10 600 python -u bench.py --image 480x640 --no-cpu-baseline > $O/bench_c1_sunrgbd.json 2> $O/bench_sun.err || fail sunbench $O/bench_sun.err
            tail -1 $O/bench_c1_sunrgbd.json | cut -c1-240 ;;
    c4parity) timeout -k 10 900 python -u tools/parity_report.py --c4-full-depth --out $O/c4_full_depth.json \
                > $O/c4_full_depth.log 2>&1 || fail c4parity $O/c4_full_depth.log ;;
    hnprofile) timeout -k 10 900 python -u tools/parity_report.py --depth-profile --out $O/depth_profile.json \
                > $O/depth_profile.log 2>&1 || fail hnprofile $O/depth_profile.log ;;
    fp8study) timeout -k 10 600 python -u tools/fp8_c4_study.py --out $O/fp8_c4.json > /dev/null 2> $O/fp8_c4.log || fail fp8study $O/fp8_c4.log
            KDSTEP_LIB=tools/ab/libkdstep_ab.so KD_GEMM_STAGGER=0 timeout -k 10 600 python -u tools/fp8_c4_study.py \
                --out $O/fp8_c4_nostagger.json > /dev/null 2> $O/fp8_c4_nostagger.log || fail fp8study-nostagger $O/fp8_c4_nostagger.log
            grep "seed" $O/fp8_c4.log $O/fp8_c4_nostagger.log ;;
    parity) timeout -k 10 600 python -u tools/parity_report.py --out $O/parity.json $PARITY_KINDS > $O/parity.log 2>&1 || fail parity $O/parity.log ;;
    ntx)    timeout -k 10 300 python -u tools/ntx_bias_study.py > $O/ntx_bias.json 2> $O/ntx_bias.err || fail ntx $O/ntx_bias.err ;;
    bench)  timeout -k 10 900 python -u bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
            tail -1 $O/bench.json | cut -c1-240 ;;
    c2|c3|c4) timeout -k 10 600 python -u bench.py --config $s --no-cpu-baseline > $O/bench_$s.json 2> $O/bench_$s.err || fail "bench $s" $O/bench_$s.err
            tail -1 $O/bench_$s.json | cut -c1-240 ;;
    ab)     IFS='|' read -ra SETS <<< "$AB_SETS"; i=0
            for v in "${SETS[@]}"; do
              i=$((i + 1))
              env $v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-delta --no-timer $AB_ARGS > $O/ab_$i.json 2> $O/ab_$i.err || fail "ab $i" $O/ab_$i.err
              python3 -c "import json; d=json.loads(open('$O/ab_$i.json').read().strip().splitlines()[-1]); print('[$v]', d['value'], d['ms_per_step'])"
            done ;;
    prof)   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --serial --no-teacher-rate --no-cpu-baseline --no-delta $BENCH_ARGS > $O/prof.log 2>&1 || fail prof $O/prof.log 20 ;;
    step)   timeout -k 10 300 rocprofv3 --kernel-trace -d $O/profstep -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-delta --no-timer --no-teacher-rate $BENCH_ARGS > $O/profstep.log 2>&1 || fail profstep $O/profstep.log 20
            DB=$(ls $O/profstep/*/run_results.db $O/profstep/run_results.db 2>/dev/null | head -1)
            python3 tools/step_breakdown.py $DB 40 > $O/step_breakdown.txt 2>&1
            python3 tools/step_phases.py $DB > $O/step_phases.txt 2>&1
            python3 tools/step_timeline.py $DB 1.0 > $O/step_timeline.txt 2>&1; head -45 $O/step_breakdown.txt ;;
    blas)   OUT=$O bash tools/pmc_vs_blas.sh > $O/pmc_blas.log 2>&1 || fail pmc_vs_blas $O/pmc_blas.log 10
            cat $O/pmc_blas/summary.txt ;;
    pmc)    OUT=$O bash tools/pmc_bench.sh > $O/pmc_bench.log 2>&1 || fail pmc $O/pmc_bench.log 10 ;;
    pmcstep) OUT=$O bash tools/pmc_bench.sh mfma > $O/pmc_step.log 2>&1 || fail pmcstep $O/pmc_step.log 10 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "done $(date +%T)"
