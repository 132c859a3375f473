"""Rank process of test_bench_launcher.test_dp_seeds_gloo: prints this rank's
shared seed and per-rank noise key."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from d3rlpy_amd.dp import DataParallel  # noqa: E402

dist.init_process_group("gloo")
rank = dist.get_rank()
torch.manual_seed(0)  # every rank seeds identically (the common user pattern)
np.random.seed(rank)  # ...but each rank's numpy draw differs
dp = DataParallel()
own = int(np.random.randint(0, 2**62))
shared = dp.shared_seed(own)
key = dp.rank_seed(int(torch.randint(0, 2**62, (1,)).item()))
print(json.dumps({"rank": rank, "own": own, "shared": shared, "key": key}), flush=True)
dist.destroy_process_group()
