set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for A in 0 1 2 4 3; do
  if [ $A = 0 ]; then L=video-gen-evals_amd/vge/libvge.so; else L=tools/abl/libvge_gabl$A.so; fi
  echo "== GABL $A"; VGE_LIB=$L timeout -k 10 120 python -u tools/gemm_bench.py --waves w8 --rounds 3 2>&1 | grep -E "tflops" || exit 1
done
