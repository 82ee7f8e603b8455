set -e
for rep in 1 2; do
  for v in dma 32 64 128; do
    if [ $v = dma ]; then export KGS_WB_COPY=dma; unset KGS_WB_BLOCKS; else unset KGS_WB_COPY; export KGS_WB_BLOCKS=$v; fi
    echo "== rep $rep wb $v"
    timeout -k 10 120 python -u profiles/host_inflight.py 20 4 48 1 device,host
  done
done
