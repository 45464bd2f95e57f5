"""torchrun worker for tests/test_bench_cpu.py (gloo on CPU): bench.py's per-rank record, its gather over the
process group and the multi-rank fields of the bench line, as main() builds them."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
dp = {"exchange": os.environ.get("FAKE_EXCHANGE", "peer"), "selftest": "pass", "error": None}
phase = {"rollout_ms": 7.0 + rank, "update_us_per_minibatch": 25.0 + rank}
rec = bench.rank_record(rank, "cpu", ("GoToPose", "TrackXYOVelocity")[rank % 2], dp, 1.2 + 0.1 * rank, 20, phase)
exchange, extra = bench.dp_fields(bench.rank_records(rec, world))
if rank == 0:
    print(json.dumps({"config": {"exchange": exchange}, "extra": extra}))
dist.barrier()
dist.destroy_process_group()
