cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for v in 0 1 0 1; do echo "== wide=$v rows=131072"; MMU_GEMM_WIDE=$v timeout -k 10 200 python -u tools/gemm_bench.py --no-ref --rows 131072 --cases "fwd o    drop,fwd ffn2,bwd dA   B=W1,bwd dX   B=Wqkv,bwd dO   B=Wo,bwd dZ   B=W2,fwd ffn1 gelu" || exit 1; done > gpurun_out/r6w_m131072.txt 2>&1
cat gpurun_out/r6w_m131072.txt | grep -v amdgpu.ids
