set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fusion_diff.py > gpurun_out/r6g_fusion_diff.log 2>&1; echo "rc $?"
cat gpurun_out/r6g_fusion_diff.log | grep -v Warning | tail -12
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "gemm_stats" 2>&1 | tail -3
