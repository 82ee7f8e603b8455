# write-combined input staging (KGS_STAGE_WC=1) vs coherent pinned staging (KGS_STAGE_WC=0, the default): single-proof
# latency by round (boundary_probe) and host-buffer proofs in flight
set -e
for rep in 1 2; do
  for v in 1 0; do
    export KGS_STAGE_WC=$v
    echo "== rep $rep KGS_STAGE_WC=$v"
    timeout -k 10 120 python -u profiles/boundary_probe.py 20 5
    timeout -k 10 120 python -u profiles/host_inflight.py 20 4 48 1 device,host
  done
done
