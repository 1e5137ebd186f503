"""Probe: bf16 eval (no_grad) ResNet trunk variants on this ROCm stack (each case in its own process)."""
import subprocess, sys
CASE = r'''
import sys, torch
sys.path.insert(0, "multi-modal-uncertainty_amd"); sys.path.insert(0, ".")
case = sys.argv[1]
from src.resnet import resnet152_trunk
import torch.nn as nn
blocks = (1,1,1,1)
x = torch.randn(2, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
if case == "plain_module_cl":
    m = resnet152_trunk(blocks).cuda().to(memory_format=torch.channels_last).eval()
elif case == "plain_module_nchw_w":
    m = resnet152_trunk(blocks).cuda().eval()
elif case == "store_views":
    from src.mmbt import MultimodalBertClf
    from src.testing import small_args
    mm = MultimodalBertClf(small_args()).cuda()
    m = mm.enc.img_encoder.model.eval()
elif case == "store_views_grad":
    from src.mmbt import MultimodalBertClf
    from src.testing import small_args
    mm = MultimodalBertClf(small_args()).cuda()
    m = mm.enc.img_encoder.model.eval()
grad = case.endswith("_grad")
for ac in [True]:
    with torch.set_grad_enabled(grad), torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
        y = m(x)
    torch.cuda.synchronize()
    print("OK", ac, y.dtype, y.stride())
'''
for case in ["plain_module_cl", "plain_module_nchw_w", "store_views", "store_views_grad"]:
    r = subprocess.run([sys.executable, "-X", "faulthandler", "-c", CASE, case], capture_output=True, text=True, timeout=300)
    tail = (r.stdout + r.stderr).strip().splitlines()
    print(f"{case:22s} rc={r.returncode} {tail[-1][:100] if tail else ''}", flush=True)
    if r.returncode != 0:
        print("\n".join(l for l in tail if "File" in l or "Error" in l)[:1500])
