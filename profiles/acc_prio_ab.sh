# Progress priority in k_accumulate (KGS_ACC_PRIO: 0 off, 1 exclusive two-lane build only = default,
# 2 every launch) against the previous library (aux kernels at priority 1, no progress priority):
# block residency alone (diag build), the lone MSM's accumulate phase, single-proof latency, in flight
set -e
D=$PWD/kzg-grandsums-study_amd/lib_ab/diag/libkgs.so
P=$PWD/kzg-grandsums-study_amd/lib_ab/prev/libkgs.so
KGS_ACC_PRIO=2 KGS_LIB=$D timeout -k 10 90 python3 -u profiles/acc_residency.py 20
for rep in 1 2; do
  for v in 0 2; do KGS_ACC_PRIO=$v timeout -k 10 90 python3 -u profiles/msm_loop.py 20 20; done
done
for rep in 1 2 3; do
  KGS_LIB=$P timeout -k 10 90 python3 -u profiles/latency_ab.py 20 15
  KGS_ACC_PRIO=1 timeout -k 10 90 python3 -u profiles/latency_ab.py 20 15
done
for rep in 1 2; do
  echo "== rep $rep prev"; KGS_LIB=$P timeout -k 10 120 python -u profiles/host_inflight.py 20 4 48 1 device
  echo "== rep $rep prio 1"; KGS_ACC_PRIO=1 timeout -k 10 120 python -u profiles/host_inflight.py 20 4 48 1 device
done
