"""Worker for tests/test_elastic.py: all-reduce once over gloo, record the world size, then idle
until the test drops a ``stop`` file (or 120 s pass)."""
import os
import sys
import time

import torch
import torch.distributed as dist

out = sys.argv[1]
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
t = torch.ones(1)
dist.all_reduce(t)
assert int(t.item()) == world
with open(os.path.join(out, f"round_w{world}_r{rank}"), "w") as f:
    f.write(os.environ["PADDLE_TRAINER_ENDPOINTS"])
dist.destroy_process_group()
t0 = time.time()
while not os.path.exists(os.path.join(out, "stop")) and time.time() - t0 < 120:
    time.sleep(0.2)
sys.exit(0)
