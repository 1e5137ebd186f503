"""Bisect the smoke-test crash: run variants of its steps, each in its own process."""
import subprocess, sys
CASE = r'''
import sys, torch
sys.path.insert(0, "multi-modal-uncertainty_amd"); sys.path.insert(0, ".")
v = sys.argv[1]
from oracle.weights import SMALL, make_state_dict
from src.mmbt import MultimodalBertClf
from src.testing import small_args, synthetic_batch
dev = torch.device("cuda:0")
if "preload" in v:
    from src import _native; _native.load()
torch.manual_seed(0)
over = dict(bert_hidden_dropout=0.0, bert_attn_dropout=0.0)
if "fp32" in v: over["img_precision"] = "fp32"
model = MultimodalBertClf(small_args(**over))
if "sd" in v:
    model.load_state_dict(make_state_dict(0, SMALL), strict=True)
model.to(dev)
x, y = synthetic_batch(2, 16, lens=[16, 9], vocab=SMALL.vocab, seed=0)
x = tuple(t.to(dev) for t in x)
if "train" in v: model.train()
else: model.eval()
with torch.set_grad_enabled("grad" in v):
    if "trunk" in v:
        f = model.enc.img_encoder.trunk(x[3])
    else:
        out = model(*x)
torch.cuda.synchronize()
print("OK")
'''
for v in ["eval", "eval_sd", "eval_sd_preload", "eval_sd_fp32", "eval_sd_grad", "train_sd_grad", "eval_sd_trunk", "eval_trunk"]:
    r = subprocess.run([sys.executable, "-X", "faulthandler", "-c", CASE, v], capture_output=True, text=True, timeout=300)
    out = (r.stdout + r.stderr).strip().splitlines()
    print(f"{v:18s} rc={r.returncode} {out[-1][:80] if out else ''}", flush=True)
    if r.returncode not in (0,):
        print("   " + "\n   ".join(l for l in out if "repo/" in l)[:800], flush=True)
