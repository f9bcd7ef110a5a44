"""A/B of the LayerNorm-backward workgroup count (SINGA_AMD_LNB_WG) on the
BERT-base shape [4096, 768] bf16: one JSON line per setting (us per call)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, torch
sys.path.insert(0, %r)
from singa_amd.ops import functional as F
x = torch.randn(4096, 768, device='cuda').bfloat16(); dy = torch.randn_like(x)
g = torch.rand(768, device='cuda') + 0.5
_, mu, rs = F.layernorm_fwd(x, g, None)
dg = torch.zeros(768, device='cuda'); db = torch.zeros(768, device='cuda')
for _ in range(5): F.layernorm_bwd(x, dy, g, mu, rs, dg_acc=dg, db_acc=db)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize(); e0.record()
for _ in range(200): F.layernorm_bwd(x, dy, g, mu, rs, dg_acc=dg, db_acc=db)
e1.record(); torch.cuda.synchronize()
print(e0.elapsed_time(e1) / 200 * 1e3)
""" % ROOT
for wg in sys.argv[1:] or ["64", "128", "256", "512", "1024"]:
    env = dict(os.environ, SINGA_AMD_LNB_WG=wg)
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=120)
    us = out.stdout.strip().splitlines()[-1] if out.returncode == 0 and out.stdout.strip() else None
    print(json.dumps({"wg": int(wg), "us": round(float(us), 2) if us else None, "rc": out.returncode}), flush=True)
