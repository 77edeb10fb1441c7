"""bench.py's config-5 measurement on its own (config5_rate: the 12.5M-key shard, HIP
events around 20 back-to-back joins), printed as one JSON line: run under rocprofv3 it
puts the bench's event-timed launch average and the profiler's kernel durations of the
SAME launches side by side (profiles/r4/c5_*)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from delta_crdt_ex_amd.store import Engine  # noqa: E402

eng = Engine(0)
r, _ = bench.config5_rate(eng, torch, torch.device("cuda", 0),
                          settle_ms=float(os.environ.get("C5_SETTLE_MS", "0")))
print(json.dumps(r), flush=True)
eng.close()
