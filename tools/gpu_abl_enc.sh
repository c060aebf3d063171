set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=video-gen-evals_amd/csrc/build
for A in 0 1 2 4 8 16 7; do
  if [ $A = 0 ]; then L=video-gen-evals_amd/vge/libvge.so; else L=$B/abl$A/libvge.so; fi
  echo "== ABL $A"; VGE_LIB=$L timeout -k 10 120 python -u tools/time_encoder.py --calls 20 --tag abl$A 2>&1 | tail -1 || exit 1
done
