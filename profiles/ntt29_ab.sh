# NTT LDS passes: twiddle products in 9 x 29-bit limbs (fr29.hpp, default) vs the 8 x 32-bit
# product-scanning product (KGS_NTT_T29=0); the transform alone (fwd+inv pairs) and the whole proof
# (device-resident, in flight), interleaved on one box
set -e
for rep in 1 2 3; do
  for v in t29 t32; do
    if [ $v = t29 ]; then unset KGS_NTT_T29; else export KGS_NTT_T29=0; fi
    echo "== rep $rep twiddle product $v"
    timeout -k 10 120 python -u profiles/ntt_ab.py 22 20
    timeout -k 10 120 python -u profiles/ntt_ab.py 20 40
    timeout -k 10 120 python -u profiles/host_inflight.py 20 4 48 1 device
  done
done
