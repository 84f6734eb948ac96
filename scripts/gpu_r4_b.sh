# round 4, GPU call B: vision tests (fused SSD tail), tail A/B, detector kernel trace, detector rel-error
# probe; ResNet-50 1x1-conv-as-GEMM A/B + step kernel table; 8-rank butterfly / ring rehearsals
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/rn50 && \
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_ps_gpu.py > gpurun_out/b_gemm_ps_tests.log 2>&1 && \
timeout -k 10 200 python -u scripts/gemm_ps_bench.py > gpurun_out/b_gemm_ps_bench.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vision_gpu.py > gpurun_out/b_vision_tests.log 2>&1 && \
timeout -k 10 120 python -u scripts/ssd_tail_ab.py > gpurun_out/b_ssd_tail_ab.log 2>&1 && \
timeout -k 10 200 bash scripts/gpu_det_prof.sh > gpurun_out/b_detprof.log 2>&1 && \
timeout -k 10 120 python -u scripts/detector_rel_err.py > gpurun_out/det_rel_err.log 2>&1 && \
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py -k "resnet or batchnorm" > gpurun_out/rn50/tests.log 2>&1 && \
for m in conv:torch gemm:fused conv:fused gemm:torch gemm:fused conv:torch; do VCX_RESNET_CONV1X1=${m%:*} VCX_RESNET_BN=${m#*:} timeout -k 10 200 python -u bench_configs.py --configs 3 --steps 10 >> gpurun_out/rn50/ab.log 2>&1 && echo "^ conv1x1:bn = $m" >> gpurun_out/rn50/ab.log || exit 1; done && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rn50/trace -o run -- \
    python3 $GRAFT_REPO_ROOT/bench_configs.py --configs 3 --steps 3 > $GRAFT_REPO_ROOT/gpurun_out/rn50/run.log 2>&1 ) && \
f=$(find gpurun_out/rn50/trace -name "*kernel_trace.csv" | head -1) && python3 scripts/prof_step_generic.py "$f" 45 > gpurun_out/rn50/step_kernels.txt && rm -f "$f"
