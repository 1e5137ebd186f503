"""Probe: which ResNet trunk precision / memory-format / mode combinations run on this ROCm stack."""
import subprocess, sys
CASE = r'''
import sys, torch
sys.path.insert(0, "multi-modal-uncertainty_amd")
from src.resnet import resnet152_trunk
fmt, dt, mode, blocks = sys.argv[1], sys.argv[2], sys.argv[3], eval(sys.argv[4])
m = resnet152_trunk(blocks).cuda()
m.train(mode == "train")
x = torch.randn(4, 3, 224, 224, device="cuda")
if fmt == "cl":
    x = x.contiguous(memory_format=torch.channels_last); m = m.to(memory_format=torch.channels_last)
if dt == "bf16w":
    m = m.to(torch.bfloat16); x = x.to(torch.bfloat16); ctx = torch.autocast("cuda", enabled=False)
else:
    ctx = torch.autocast("cuda", dtype=torch.bfloat16, enabled=(dt == "autocast"))
with ctx:
    y = m(x)
    if mode == "train":
        y.float().sum().backward()
torch.cuda.synchronize()
print("OK", y.dtype, y.shape, y.stride())
'''
for blocks in ["(1,1,1,1)", "(3,8,36,3)"]:
    for fmt in ["cl", "nchw"]:
        for dt in ["autocast", "bf16w", "fp32"]:
            for mode in ["eval", "train"]:
                r = subprocess.run([sys.executable, "-c", CASE, fmt, dt, mode, blocks], capture_output=True, text=True, timeout=300)
                last = (r.stdout.strip().splitlines() or [""])[-1]
                print(f"{blocks:12s} {fmt:5s} {dt:9s} {mode:5s} rc={r.returncode} {last[:80]}", flush=True)
