# round 4, GPU call Q: BASELINE configs 3 (ResNet-50 + top-k), 4 (GPT-2-medium) and 5 (Llama-3-8B sharded +
# PowerSGD, one peer) on the final tree, one GPU.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/q || exit 1
timeout -k 10 900 python -u bench_configs.py --configs 3,4,5 --steps 8 > gpurun_out/q/configs.log 2>&1
echo "rc=$?" >> gpurun_out/q/configs.log
