set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2 3 4; do
for ov in 0 1; do
VGE_FLOW_OVERLAP=$ov timeout -k 10 300 python -u bench.py --workload tag --steps 10 --warmup 2 > gpurun_out/bench_tag_ov$ov.log 2>&1 || exit 1
echo "overlap=$ov $(tail -1 gpurun_out/bench_tag_ov$ov.log | grep -o '"value": [0-9.]*')"
done; done
