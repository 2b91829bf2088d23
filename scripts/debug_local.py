"""Debug: Local generate vs teacher-forced forward on the clone case (graph vs direct)."""
import os, sys, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_local_gpu import make_local_engine, lcase
from oracle import moss_local as L
g = np.load("tests/golden/golden_local.npz")
cases = json.load(open("tests/golden/cases_local.json"))
name = sys.argv[1] if len(sys.argv) > 1 else "l_nvq8_clone_bf16"
gg, c, cfg, W = lcase((g, cases), name)
ids, ref = g[name + "/input_ids"], g[name + "/out"]
T = ids.shape[1]
eng = make_local_engine(cfg, W)
out = eng.local_generate_ids(torch.from_numpy(ids), None, 3, c["n_vq_inf"]).cpu().numpy()
print("gen  f0", out[:, T].tolist()); print("ref  f0", ref[:, T].tolist())
print("gen  f1", out[:, T + 1].tolist()); print("ref  f1", ref[:, T + 1].tolist())
# teacher-forced frame 1 with our own frame 0 / frame 1
x = out[:, T:T + 1].copy()
mask = np.ones((ids.shape[0], T + 1), np.uint8)
lg = eng.local_forward(torch.from_numpy(x), torch.from_numpy(mask), T, torch.from_numpy(out[:, T + 1].copy()), c["n_vq_inf"])
print("fwd  f1", np.stack([t.float().argmax(-1).cpu().numpy() for t in lg], -1).tolist())
