# k_accumulate block residency alone, from the diagnostic build's block stamps:
#   make -C kzg-grandsums-study_amd EXTRA=-DKGS_DIAG_CLOCK BUILD=build_diag LIBOUT=lib_ab/diag/libkgs.so lib_ab/diag/libkgs.so
# (lib_diag/ is gpurun-ignored; lib_ab/ travels). KGS_ACC_PRIO=0 / 2: progress priority off / on for this launch
set -e
D=$PWD/kzg-grandsums-study_amd/lib_ab/diag/libkgs.so
KGS_ACC_PRIO=0 KGS_LIB=$D timeout -k 10 90 python3 -u profiles/acc_residency.py 20
KGS_ACC_PRIO=2 KGS_LIB=$D timeout -k 10 90 python3 -u profiles/acc_residency.py 20
