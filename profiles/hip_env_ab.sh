# Single-proof host-buffer latency under the HIP runtime the JS module binds to (/opt/rocm 7.2, no
# torch in the process) with runtime knobs, against torch's bundled 7.0 runtime; same box, interleaved
# usage: bash profiles/hip_env_ab.sh [reps=3]
set -e
for rep in $(seq 1 ${1:-3}); do
  for v in torch notorch kernarg1 kernarg0 blit; do
    unset HIP_FORCE_DEV_KERNARG ROC_SKIP_KERNEL_ARG_COPY HIP_FORCE_BLIT_COPY
    mode=notorch
    case $v in
      torch) mode=torch ;;
      kernarg1) export HIP_FORCE_DEV_KERNARG=1 ;;
      kernarg0) export HIP_FORCE_DEV_KERNARG=0 ;;
      blit) export ROC_SKIP_KERNEL_ARG_COPY=1 ;;
    esac
    echo "== rep $rep $v"
    timeout -k 10 120 python -u profiles/hip_runtime_ab.py $mode 20 9 | grep -E "median" | tail -1
  done
done
