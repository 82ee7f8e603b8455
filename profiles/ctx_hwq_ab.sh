# host-buffer vs device-resident in flight: contexts x hardware queues (GPU_MAX_HW_QUEUES)
set -e
for rep in 1 2; do
  for q in 4 8; do
    export GPU_MAX_HW_QUEUES=$q
    echo "== rep $rep hw queues $q"
    timeout -k 10 200 python -u profiles/host_inflight.py 20 4,6,8 48 1 device,host
  done
done
