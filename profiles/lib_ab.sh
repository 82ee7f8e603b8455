# Same-box A/B of the in-tree library against kzg-grandsums-study_amd/lib_ab/<variant>/libkgs.so (the
# previous commit's build, or a -D variant built with the Makefile's EXTRA/BUILD/LIBOUT): proofs in
# flight, device-resident, interleaved reps
# usage: bash profiles/lib_ab.sh [reps=3] [variant=prev]
set -e
VAR=${2:-prev}
for rep in $(seq 1 ${1:-3}); do
  for v in new $VAR; do
    if [ $v = new ]; then unset KGS_LIB; else export KGS_LIB=$PWD/kzg-grandsums-study_amd/lib_ab/$VAR/libkgs.so; fi
    echo "== rep $rep library $v"
    timeout -k 10 120 python -u profiles/host_inflight.py 20 4 48 1 device
  done
done
