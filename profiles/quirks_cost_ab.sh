# cost of reference-quirks detection (KGS_REFERENCE_QUIRKS=1: degree kernels of the base operands and
# a zero-quotient check, one host round trip each) on the headline workload, interleaved, same box
set -e
for rep in 1 2; do
  for v in 0 1; do
    export KGS_REFERENCE_QUIRKS=$v
    echo "== rep $rep KGS_REFERENCE_QUIRKS=$v"
    timeout -k 10 120 python -u profiles/host_inflight.py 20 4 64 1 device
  done
done
for v in 0 1; do
  export KGS_REFERENCE_QUIRKS=$v
  echo "== latency KGS_REFERENCE_QUIRKS=$v"
  timeout -k 10 120 python -u profiles/boundary_probe.py 20 7 2>&1 | grep "^device"
done
