#!/bin/bash
# round 6: NTT passes on 2^12-element tiles (-DKGS_NTT_ELOG=12: 128 KiB LDS, 512 threads, up to 12
# stages per pass: 2^21 = 9+12, two global round trips instead of three) against the in-tree 2^11
# tiles. Parity of the variant first (NTT 2^0..2^22 vs the oracles, golden proofs, 2^20 proof byte-exact),
# then the fwd+inv pair alone and the proofs in flight, interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/ntt_e12
mkdir -p $O
export PYTHONUNBUFFERED=1
E12=$PWD/kzg-grandsums-study_amd/lib_ab/e12/libkgs.so
KGS_LIB=$E12 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "test_ntt or test_golden_proofs or test_c1_grandsum_2p20_exact" \
  > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -3 $O/parity.log
for rep in 1 2 3; do
  for v in e11 e12 e12d; do
    case $v in
      e11) unset KGS_LIB KGS_NTT_DIRECT_TILE ;;
      e12) export KGS_LIB=$E12; unset KGS_NTT_DIRECT_TILE ;;
      e12d) export KGS_LIB=$E12 KGS_NTT_DIRECT_TILE=1 ;;
    esac
    for lg in 21 20 22; do
      timeout -k 10 120 python -u profiles/ntt_ab.py $lg 20 2>&1 | sed "s/^/rep $rep $v /" || exit 1
    done
  done
done | tee $O/pair_ab.txt
for rep in 1 2; do
  for v in e11 e12; do
    if [ $v = e11 ]; then unset KGS_LIB; else export KGS_LIB=$E12; fi
    unset KGS_NTT_DIRECT_TILE
    echo "== rep $rep $v"
    timeout -k 10 120 python -u profiles/host_inflight.py 20 4 48 1 device || exit 1
  done
done 2>&1 | tee $O/inflight_ab.txt
