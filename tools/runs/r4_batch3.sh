# round 4 lease 3: ViLT / encoders, the DP tests after the side-stream routing change, the dropout
# joint-statistics test, then the attention A/B (ab/maskskip.so, ab/w3.so vs the committed library)
set -o pipefail
mkdir -p gpurun_out
bash tools/runs/r4_vilt.sh || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_dp_gpu.py tests/test_mmbt_gpu.py -q -s --timeout 300 --timeout-method thread -k "dp or side_stream" > gpurun_out/r4_dp_tests.log 2>&1 || { tail -30 gpurun_out/r4_dp_tests.log; exit 1; }
grep -E "dp parity|passed|failed" gpurun_out/r4_dp_tests.log
MMU_LIB_PATH=ab/w3.so timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -q -s --timeout 200 --timeout-method thread -k "joint_statistics" > gpurun_out/r4_dropjoint.log 2>&1 || { tail -30 gpurun_out/r4_dropjoint.log; exit 1; }
grep -E "dropout joint|passed|failed" gpurun_out/r4_dropjoint.log
bash tools/runs/r4_maskskip.sh
