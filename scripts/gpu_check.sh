#!/bin/bash
# One bounded GPU session: kernel tests -> engine tests -> short bench. Stops after any
# fault-type exit (abort/segv/timeout); plain test failures (rc=1) continue.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc[$name]=$rc"; tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
python -c "import torch;print(torch.cuda.get_device_name(0), torch.cuda.mem_get_info())"
for s in "$@"; do
  case $s in
    kernels) step kernels 900 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x ;;
    engine)  step engine 900 python -m pytest tests/test_engine_gpu.py -q -m gpu -x ;;
    gputests) step gputests 1200 python -m pytest tests -q -m gpu ;;
    smoke)   step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   step bench 900 python bench.py --steps 2 --warmup 1 ;;
    reference) step reference 900 python scripts/bench_reference.py --out gpurun_out/reference_strategy.json ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 1 --warmup 1
          python scripts/prof_summary.py gpurun_out/prof 40 --tail-ms 900 > gpurun_out/prof_summary.txt
          rm -f gpurun_out/prof/*trace.csv ;;
    prof_noblas) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          step prof_noblas 900 env DLI_GEMM_NO_BLAS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_noblas -o bench -- python bench.py --steps 1 --warmup 1
          python scripts/prof_summary.py gpurun_out/prof_noblas 40 --tail-ms 900 > gpurun_out/prof_noblas_summary.txt
          rm -f gpurun_out/prof_noblas/*trace.csv ;;
    prof_mixtral) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          step prof_mixtral 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mixtral -o bench -- python bench.py --model mixtral-8x7b --steps 1 --warmup 1 --batch 512
          python scripts/prof_summary.py gpurun_out/prof_mixtral 40 --tail-ms 4000 > gpurun_out/prof_mixtral_summary.txt
          rm -f gpurun_out/prof_mixtral/*trace.csv ;;
    pp2) step pp2 900 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --batch 64 ;;
    pp4) step pp4 900 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 1 --warmup 1 --batch 32 ;;
    pp8) step pp8 900 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 8 --steps 1 --warmup 1 --batch 16 ;;
    nccl1) step nccl1_pp 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 2 --mode pp --steps 1 --warmup 1 --batch 64
           step nccl1_dp 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 2 --mode dp --steps 1 --warmup 1 --batch 64 ;;
    gemm) step gemm 1100 python scripts/bench_gemm.py ;;
    ops) step ops 600 python scripts/bench_ops.py ;;
    ab) step ab_fused 600 python bench.py --steps 2 --warmup 1
        step ab_unfused 600 env DLI_NO_FUSED_REDUCE=1 python bench.py --steps 2 --warmup 1
        step ab_notune 600 env DLI_GEMM_AUTOTUNE=0 python bench.py --steps 2 --warmup 1
        step ab_fused2 600 python bench.py --steps 2 --warmup 1 ;;
    mixtral1) step mixtral1 900 python bench.py --model mixtral-8x7b --steps 1 --warmup 1 --batch 128 ;;
    ep4) step ep4 900 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29539 bench.py --model mixtral-8x7b --gpus 4 --steps 1 --warmup 1 --batch 32 ;;
    ep2) step ep2 900 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --model mixtral-8x7b --gpus 2 --steps 1 --warmup 1 --batch 32 ;;
    llama70) step llama70 1100 python bench.py --model llama3-70b --steps 1 --warmup 1 --batch 64 ;;
    bench_small) step bench_small 600 python bench.py --steps 2 --warmup 1 --batch 64 ;;
    b1) step bench_b1 600 python bench.py --steps 16 --warmup 2 --batch 1 ;;
    prof8k) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          step prof8k 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof8k -o bench -- python bench.py --steps 1 --warmup 1 --batch 1 --prompt-len 8064 --max-length 8180 --max-model-len 8192
          python scripts/prof_summary.py gpurun_out/prof8k 40 --tail-ms 250 > gpurun_out/prof8k_summary.txt
          rm -f gpurun_out/prof8k/*trace.csv ;;
    lookahead) step la_on 600 python bench.py --steps 3 --warmup 1
               step la_off 600 env DLI_LOOKAHEAD=0 python bench.py --steps 3 --warmup 1
               step la_on2 600 python bench.py --steps 3 --warmup 1 ;;
    engine_tests) step engine_tests 900 python -u -m pytest tests/test_engine_gpu.py tests/test_lookahead.py -x -v --timeout 300 --timeout-method thread ;;
    noblas) step noblas 900 env DLI_GEMM_AUTOTUNE_LOG=1 python bench.py --steps 2 --warmup 1
            step withblas 900 env DLI_GEMM_DECODE_BLAS=1 DLI_GEMM_AUTOTUNE_LOG=1 python bench.py --steps 2 --warmup 1 ;;
    tune) step tune_off 600 python bench.py --steps 2 --warmup 1
          step tune_on 900 env DLI_GEMM_AUTOTUNE=1 DLI_GEMM_AUTOTUNE_LOG=1 python bench.py --steps 2 --warmup 1
          step tune_on256 900 env DLI_GEMM_AUTOTUNE=1 python bench.py --steps 2 --warmup 1 --batch 256 ;;
    sweep) for b in 128 384 512 768; do
             step sweep_b$b 600 python bench.py --steps 2 --warmup 1 --batch $b
           done ;;
    moe_tiles) for t in 12 10; do
             step moe_tile$t 900 env DLI_MOE_TILE=$t python bench.py --model mixtral-8x7b --steps 1 --warmup 1 --batch 512
           done ;;
    moe_tuned) for b in 128 512; do
             step moe_tuned_b$b 900 env DLI_GEMM_AUTOTUNE_LOG=1 python bench.py --model mixtral-8x7b --steps 1 --warmup 1 --batch $b
           done ;;
    mixtral_sweep) for b in 256 512; do
             step mixtral_b$b 900 python bench.py --model mixtral-8x7b --steps 1 --warmup 1 --batch $b
           done ;;
    llama70b) for b in 128 256; do
             step llama70_b$b 900 python bench.py --model llama3-70b --steps 1 --warmup 1 --batch $b
           done ;;
  esac
done
