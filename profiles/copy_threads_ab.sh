# host-buffer in flight vs the host threads of the staging copies (KGS_COPY_THREADS); the box's CPU share
set -e
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)  nproc: $(nproc)  allowed: $(grep Cpus_allowed_list /proc/self/status)"
for rep in 1 2; do
  for v in 16 8 4; do
    export KGS_COPY_THREADS=$v
    echo "== rep $rep copy threads $v"
    timeout -k 10 120 python -u profiles/host_inflight.py 20 4 48 1 device,host
  done
done
