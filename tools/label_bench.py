"""Time rs_staytime_labels at the config-5 batch (16384 per step, staytime/parse.py:16-71):
HIP events on the launch stream; algorithmic bytes/sample = 8 (watch ms) + 1 (landing) +
4 * 401 (soft label ++ seconds) + 12 (short, long, weight) = 1625 B."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from recommendsystem_amd.parse import staytime_labels  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
rng = np.random.default_rng(0)
wt = torch.from_numpy(np.exp(rng.normal(9.5, 1.5, size=B)).astype(np.int64)).cuda()
land = torch.from_numpy((rng.uniform(size=B) < 0.1).astype(np.uint8)).cuda()
for _ in range(10):
    staytime_labels(wt, land)
reps = 200
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    staytime_labels(wt, land)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / reps
print(json.dumps({"B": B, "us_per_call": round(us, 2), "GB/s": round(B * 1625 / us / 1e3, 1)}))
