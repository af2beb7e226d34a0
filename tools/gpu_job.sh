#!/bin/bash
# One parameterised GPU job (replaces the per-experiment gpu_r3_*.sh
# launchers).  Each argument is a step; steps run in order under their own
# time limit (tools/gpu_step.sh) and the job stops at the first fault,
# abort, segfault or timeout.  Logs go to gpurun_out/<step>.log.
#
#   tools/gpu_job.sh STEP [STEP ...]
#
# steps:
#   tests[:PATTERN]          pytest -m gpu (PATTERN: test file(s) or -k expr,
#                            e.g. tests:tests/test_gemm_t4_gpu.py)
#   smoke                    __graft_entry__.smoke()
#   bench[:ARGS]             python bench.py ARGS (comma-separated, e.g.
#                            bench:--batch,512,--model,vgg16)
#   benv:VAR=VAL[+VAR=VAL][:ARGS]  bench.py under extra environment settings
#                            (A/B of whole steps, e.g. benv:VELES_AMD_GEMM_VARIANT=50)
#   solo[:ARGS]              bench.py with a one-rank RCCL process group
#                            (VELES_AMD_DP_SOLO_COLLECTIVES=1)
#   ab[:B:ROUNDS:VARIANTS]   tools/bench_gemm_ab.py (GEMM loop A/B)
#   abenv:VAR=VAL[+VAR=VAL]:B:ROUNDS:VARIANTS  the same under extra environment
#                            settings (e.g. HVK_LIBRARY=build/abl/libhvk_abl1.so,
#                            a tools/build_abl.py diagnostic build)
#   prof[:MODEL:BATCH:TAG:PREC]  step-only rocprofv3 kernel table
#   profenv:VAR=VAL[+VAR=VAL]:MODEL:BATCH:TAG:PREC  the same under extra
#                            environment settings (set before rocprofv3)
#   pmc[:TAG[:BENCHARGS]]    four rocprofv3 --pmc passes (instruction mix,
#                            wave states, HBM read + TA, HBM write + L2 hit)
#                            on bench.py --mark-steps, step-only summaries
#   py:SCRIPT[,ARGS]         python SCRIPT ARGS
#   rocprof:TAG:SCRIPT[,ARGS]  rocprofv3 --kernel-trace of python3 SCRIPT ARGS
#                            into gpurun_out/rp_TAG (csv)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=""
  [ "$kind" != "$step" ] && arg=${step#*:}
  log=gpurun_out/job${n}_${kind}.log
  echo "[gpu_job] step $n: $step -> $log"
  case $kind in
    tests)
      sel=${arg:-tests}
      tools/gpu_step.sh 900 "$log" python -u -m pytest $sel -m gpu -v \
        --timeout 200 --timeout-method thread -x || exit 1
      tail -3 "$log"
      grep -E "FAILED|ERROR" "$log" | head -20 ;;
    smoke)
      tools/gpu_step.sh 300 "$log" python -c \
        "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
      tail -2 "$log" ;;
    bench)
      tools/gpu_step.sh 600 "$log" python bench.py ${arg//,/ } || exit 1
      grep metric "$log" || tail -5 "$log" ;;
    benv)
      IFS=: read -r envs bargs <<< "$arg"
      tools/gpu_step.sh 600 "$log" env ${envs//+/ } python bench.py ${bargs//,/ } || exit 1
      echo "$envs"; grep metric "$log" || tail -5 "$log" ;;
    solo)
      tools/gpu_step.sh 600 "$log" env VELES_AMD_DP_SOLO_COLLECTIVES=1 \
        python bench.py ${arg//,/ } || exit 1
      grep metric "$log" || tail -5 "$log" ;;
    ab)
      IFS=: read -r b rounds vars <<< "$arg"
      tools/gpu_step.sh 900 "$log" python -u tools/bench_gemm_ab.py \
        "${b:-1024}" "${rounds:-3}" "${vars:--1}" || exit 1
      cat "$log" | head -60 ;;
    profenv)
      IFS=: read -r envs m b tag prec <<< "$arg"
      M=${m:-alexnet} B=${b:-2048} T=${tag:-r4} P=${prec:-bfloat16}
      tools/gpu_step.sh 600 "$log" env ${envs//+/ } rocprofv3 --kernel-trace \
        --stats -d "$R/gpurun_out/prof_${M}_${T}" -o run --output-format csv -- \
        python3 "$R/bench.py" --model $M --precision $P --steps 5 \
        --warmup 2 --batch $B --mark-steps || exit 1
      f=$(find gpurun_out/prof_${M}_${T} -name "*kernel_trace.csv" | head -1)
      python tools/prof_summary.py "$f" gpurun_out/prof_${M}_${T}.md \
        "$M b$B 1x MI355X ($P, $T, $envs)" --window --steps 5
      head -40 gpurun_out/prof_${M}_${T}.md ;;
    abenv)
      IFS=: read -r envs b rounds vars <<< "$arg"
      tools/gpu_step.sh 900 "$log" env ${envs//+/ } python -u \
        tools/bench_gemm_ab.py "${b:-1024}" "${rounds:-3}" "${vars:--1}" || exit 1
      echo "$envs"; cat "$log" | head -60 ;;
    prof)
      IFS=: read -r m b tag prec <<< "$arg"
      M=${m:-alexnet} B=${b:-1024} T=${tag:-r4} P=${prec:-bfloat16}
      tools/gpu_step.sh 600 "$log" rocprofv3 --kernel-trace --stats \
        -d "$R/gpurun_out/prof_${M}_${T}" -o run --output-format csv -- \
        python3 "$R/bench.py" --model $M --precision $P --steps 5 \
        --warmup 2 --batch $B --mark-steps || exit 1
      f=$(find gpurun_out/prof_${M}_${T} -name "*kernel_trace.csv" | head -1)
      python tools/prof_summary.py "$f" gpurun_out/prof_${M}_${T}.md \
        "$M b$B 1x MI355X ($P, $T)" --window --steps 5
      head -40 gpurun_out/prof_${M}_${T}.md ;;
    pmc)
      IFS=: read -r tag bargs <<< "$arg"
      T=${tag:-r4}
      for pass in A B C D; do
        case $pass in
          A) ctr="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16" ;;
          B) ctr="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" ;;
          C) ctr="FETCH_SIZE TA_BUSY_avr GRBM_GUI_ACTIVE" ;;
          D) ctr="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" ;;
        esac
        tools/gpu_step.sh 200 gpurun_out/pmc_${T}_$pass.log timeout -s KILL 150 \
          rocprofv3 --kernel-trace --pmc $ctr -d "$R/gpurun_out/pmc_${T}_$pass" \
          -o run --output-format csv -- python3 "$R/bench.py" --steps 2 \
          --warmup 2 --mark-steps ${bargs//,/ } || exit 1
      done
      f() { find gpurun_out/pmc_${T}_$1 -name "*counter_collection.csv" | head -1; }
      python tools/pmc_mix_summary.py --window "$(f A)" "$(f B)" \
        gpurun_out/pmc_mix_$T.md "step kernels: instruction mix and wave states ($T)"
      python tools/pmc_mem_summary.py --window "$(f C)" "$(f D)" \
        gpurun_out/pmc_mem_$T.md "step kernels: HBM traffic, L2 hit rate, TA busy ($T)"
      head -30 gpurun_out/pmc_mix_$T.md; head -30 gpurun_out/pmc_mem_$T.md ;;
    py)
      tools/gpu_step.sh 900 "$log" python -u ${arg//,/ } || exit 1
      tail -40 "$log" ;;
    rocprof)
      IFS=: read -r tag script <<< "$arg"
      tools/gpu_step.sh 600 "$log" rocprofv3 --kernel-trace \
        -d "$R/gpurun_out/rp_$tag" -o run --output-format csv -- \
        python3 ${script//,/ } || exit 1
      find gpurun_out/rp_$tag -name "*kernel_trace.csv" | head -1 ;;
    *)
      echo "[gpu_job] unknown step $step"; exit 2 ;;
  esac
done
