# host-buffer in flight: copy streams at low priority (own hardware-queue pool, default) vs normal
# priority, and normal priority with 16 hardware queues; device-resident beside each
set -e
for rep in 1 2 3; do
  for v in low normal normal_hwq16; do
    unset GPU_MAX_HW_QUEUES
    if [ $v = low ]; then unset KGS_COPY_STREAM_PRIO; else export KGS_COPY_STREAM_PRIO=normal; fi
    if [ $v = normal_hwq16 ]; then export GPU_MAX_HW_QUEUES=16; fi
    echo "== rep $rep copy streams $v"
    timeout -k 10 120 python -u profiles/host_inflight.py 20 4 48 1 device,host
  done
done
