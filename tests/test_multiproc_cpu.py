"""The N>1 path of bench.py / batch drivers (gsnapdp.shard) on CPU: two ranks
under the gloo backend, each aligning its own shard with the CPU restatement
(the GPU step's stand-in here), timed by the same barrier + max-over-ranks
code the benchmark uses."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from gsnapdp import shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, outdir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import oracle as O
    from gsnapdp import shard as S
    from gsnapdp import workload as W

    r = S.init_from_env("gloo")
    genome = W.synthetic_genome(300_000, seed=1)
    blocks = W.pack_genome(genome)
    batch = W.c2_windows(genome, n=300, seed=S.shard_seed(2, r.rank))
    O.setup(blocks)
    out = {}

    def step():
        res, _, _, _ = O.run_batch(batch.windows, batch.query, batch.query_uc, nthreads=1)
        out["score_sum"] = int(res["finalscore"].astype(np.int64).sum())

    elapsed = S.timed_steps(r, step, 2, lambda: None)
    rate = S.aggregate_rate(len(batch), r, 2, elapsed)
    # every rank must see the same (max) time; shards must differ
    t = torch.tensor([elapsed], dtype=torch.float64)
    ts = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    r.dist.all_gather(ts, t)
    first = torch.tensor([int(batch.windows["chrpos"][0])], dtype=torch.int64)
    firsts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    r.dist.all_gather(firsts, first)
    total = torch.tensor([len(batch)], dtype=torch.int64)
    r.dist.all_reduce(total)
    json.dump({"elapsed": [float(x) for x in ts], "firsts": [int(x) for x in firsts],
               "total": int(total), "rate": rate, "score_sum": out["score_sum"]},
              open(os.path.join(outdir, "rank%d.json" % r.rank), "w"))
    S.finish(r)


def test_shard_range_covers_batch_exactly():
    for n in (0, 1, 7, 100, 101):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(n, r, world) for r in range(world)]
            covered = [i for lo, hi in spans for i in range(lo, hi)]
            assert covered == list(range(n))


def test_single_rank_needs_no_process_group(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    r = shard.init_from_env("gloo")
    assert (r.rank, r.world, r.dist) == (0, 1, None)
    assert shard.timed_steps(r, lambda: None, 3, lambda: None) >= 0.0
    assert shard.aggregate_rate(100, r, 2, 0.5) == 400.0


@pytest.mark.timeout(300)
def test_two_ranks_gloo(tmp_path):
    world = 2
    mp.spawn(_rank_main, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [json.load(open(os.path.join(str(tmp_path), "rank%d.json" % r))) for r in range(world)]
    # max-over-ranks timing: identical on every rank
    assert res[0]["elapsed"] == res[1]["elapsed"]
    assert max(res[0]["elapsed"]) == min(res[0]["elapsed"])
    # disjoint shards (different seeds), whole-job unit count and rate
    assert res[0]["firsts"][0] != res[0]["firsts"][1]
    assert res[0]["total"] == 600
    el = res[0]["elapsed"][0]
    assert abs(res[0]["rate"] - 600 * 2 / el) < 1e-6 * res[0]["rate"]
    assert res[0]["score_sum"] != res[1]["score_sum"]
