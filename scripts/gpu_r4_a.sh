# round 4, GPU call A: gemm_ps tests + store diagnostics, attention forward v2 A/B, 8-rank direct bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_ps_gpu.py > gpurun_out/a_gemm_ps_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/gemm_ps_diag.py > gpurun_out/a_gemm_ps_diag.log 2>&1 && \
timeout -k 10 240 python -u scripts/attn_variants.py > gpurun_out/a_attn_variants.log 2>&1 && \
ONLY="bench_n8_direct" timeout -k 10 500 bash scripts/gpu_rccl8_rehearsal.sh
