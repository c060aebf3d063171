cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/ab_libs.sh 3 rot0 default xcd3 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_xcd3.log
cd /tmp && export TMPDIR=/tmp
for v in rot0 xcd3 default; do
  case $v in default) L=$GRAFT_REPO_ROOT/video-gen-evals_amd/vge/libvge.so;; *) L=$GRAFT_REPO_ROOT/video-gen-evals_amd/csrc/build/$v/libvge.so;; esac
  VGE_LIB=$L timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcx_$v -o run -- python3 $GRAFT_REPO_ROOT/tools/time_encoder.py --calls 6 --tag $v > $GRAFT_REPO_ROOT/gpurun_out/pmcx_$v.log 2>&1 || exit 1
done
cat $GRAFT_REPO_ROOT/gpurun_out/ab_xcd3.log
