# bitwise A/B of library builds on tools/ab_bits.py's scenes:
#   bash tools/gpu_bits.sh "LIB_A LIB_B [LIB_C ...]" [SCENE ...]   (each compared with LIB_A)
set -o pipefail
LIBS=$1; shift
for L in $LIBS; do
  GSR_LIBRARY=$PWD/build_var/libgsr_$L.so timeout -k 10 200 python3 tools/ab_bits.py gpurun_out/b_$L.npz "$@" > /dev/null || exit 1
done
A=${LIBS%% *}
for L in ${LIBS#* }; do echo "== $A vs $L"; python3 tools/ab_bits.py --cmp gpurun_out/b_$A.npz gpurun_out/b_$L.npz; done
exit 0
