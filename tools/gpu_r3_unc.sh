# uncertainty path after the batched residual-LayerNorm recompute: parity tests, then the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_uncertainty_gpu.py "tests/test_kernels_gpu.py::test_gemm_residual_recomputed_layernorm" -x -v --timeout 300 --timeout-method thread > gpurun_out/t_unc.log 2>&1 || { tail -40 gpurun_out/t_unc.log; exit 1; }
tail -3 gpurun_out/t_unc.log
timeout -k 10 400 python3 -u bench.py --workload uncertainty --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_unc.log 2>&1 || { tail -30 gpurun_out/b_unc.log; exit 1; }
tail -2 gpurun_out/b_unc.log
