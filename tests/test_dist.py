"""Multi-rank path on CPU: world_size-2 gloo processes run bench's sharding and
reductions (lzma-sdk-zliblike_amd/dist_bench.py).  Each rank decodes its shard
with the oracle (the GPU decoder runs the same shards on the box); together
the shards must cover the batch exactly once and reproduce the plaintext."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "lzma-sdk-zliblike_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import lzma
    import torch.distributed as dist
    import dist_bench as D
    import native
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, r, lr = D.world_info()
        assert (w, r, lr) == (world, rank, rank)
        total = 37
        lens = [100 + 97 * i for i in range(total)]
        start, count = D.shard_by_weight(lens, world, rank)
        s2, c2 = D.shard(total, world, rank)
        orc = native.oracle()
        ok = True
        for i in range(start, start + count):
            data = native.gen("text", 9000 + i, lens[i])
            f = [{"id": lzma.FILTER_LZMA1, "dict_size": 1 << 16, "lc": 3, "lp": 0, "pb": 2}]
            c = lzma.compress(data, format=lzma.FORMAT_RAW, filters=f)
            res = native.decode(orc, "orc", c, b"\x5d\x00\x00\x01\x00", lens[i], 1)
            ok = ok and res[0] == 0 and res[4] == data
        D.barrier()
        elapsed = D.reduce_max(1.0 + rank)
        nbytes = D.reduce_sum(float(sum(lens[start:start + count])))
        all_ok = D.all_true(ok)
        some_false = D.all_true(rank == 0)
        q.put((rank, start, count, s2, c2, elapsed, nbytes, all_ok, some_false))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sharding_and_reductions():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lens = [100 + 97 * i for i in range(37)]
    covered = []
    for rank, start, count, s2, c2, elapsed, nbytes, all_ok, some_false in out:
        covered += list(range(start, start + count))
        assert elapsed == float(world)          # MAX over ranks
        assert nbytes == float(sum(lens))       # SUM over ranks
        assert all_ok and not some_false       # MIN of flags
    assert covered == list(range(37))           # weight shards: exactly once, in order
    eq = [(s2, c2) for _, _, _, s2, c2, *_ in out]
    assert eq == [(0, 19), (19, 18)]


def _scatter_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "lzma-sdk-zliblike_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import lzma
    import torch
    import torch.distributed as dist
    import dist_bench as D
    import native
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # config-4 shape: rank 0 holds an LZMA2 stream of dict-reset blocks
        # (the MT-encoder layout) and scatters each rank's block range
        per_rank, plain = 3, [native.gen("text", 4400 + i, 20000 + 777 * i) for i in range(6)]
        f = [{"id": lzma.FILTER_LZMA2, "dict_size": 1 << 16, "lc": 3, "lp": 0, "pb": 2}]
        comps = [lzma.compress(b, format=lzma.FORMAT_RAW, filters=f)[:-1] for b in plain]
        offs = [0]
        for c in comps:
            offs.append(offs[-1] + len(c))
        ranges = [(offs[r * per_rank], offs[(r + 1) * per_rank]) for r in range(world)]
        src = torch.frombuffer(bytearray(b"".join(comps)), dtype=torch.uint8) if rank == 0 else None
        lo, hi = ranges[rank]
        out = torch.empty(hi - lo, dtype=torch.uint8)
        D.scatter_ranges(src, ranges, out, rank, world)
        mine = out.numpy().tobytes()
        orc = native.oracle()
        ok, decoded = True, []
        for k in range(per_rank):
            b = rank * per_rank + k
            blk = mine[offs[b] - lo:offs[b + 1] - lo]
            res, st, dl, sl, data = native.lzma2_decode(orc, "orc", blk, 16, len(plain[b]), 0)
            ok = ok and (res, st, dl, sl) == (0, 2, len(plain[b]), len(blk)) and data == plain[b]
            decoded.append(data)
        # the optional last step: every rank's decoded blocks gathered on rank 0
        dec = b"".join(decoded)
        sizes = [sum(len(plain[r * per_rank + k]) for k in range(per_rank)) for r in range(world)]
        whole = torch.empty(sum(sizes), dtype=torch.uint8) if rank == 0 else None
        D.gather_ranges(torch.frombuffer(bytearray(dec), dtype=torch.uint8), sizes, whole, rank,
                        world)
        if rank == 0:
            ok = ok and whole.numpy().tobytes() == b"".join(plain)
        q.put((rank, len(mine), ok))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_lzma2_block_scatter_and_gather():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok and n > 0 for _, n, ok in out)


def test_shard_helpers_single_process():
    sys.path.insert(0, os.path.join(ROOT, "lzma-sdk-zliblike_amd"))
    import dist_bench as D
    for total in (0, 1, 7, 65536):
        for world in (1, 2, 3, 8):
            got = [D.shard(total, world, r) for r in range(world)]
            assert sum(c for _, c in got) == total
            assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(world - 1))
    w = [1, 1, 1, 100, 1, 1]
    parts = [D.shard_by_weight(w, 2, r) for r in range(2)]
    assert parts[0][0] == 0 and parts[0][0] + parts[0][1] == parts[1][0]
    assert parts[1][0] + parts[1][1] == len(w)


def _bench_line(cmd):
    import json
    import subprocess
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints ONE JSON line
    return json.loads(lines[0])


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_bench_gpus_flag_spawns_ranks(scaling):
    """`bench.py --gpus 2` on its own starts 2 rank processes (RANK/WORLD_SIZE set
    before any GPU call) and reports n_gpus = 2; --dry-run runs the launcher,
    sharding and reductions on gloo without decoding."""
    line = _bench_line([sys.executable, "bench.py", "--gpus", "2", "--dry-run", "--steps", "2",
                        "--scaling", scaling])
    assert line["n_gpus"] == 2 and line["world"] == 2 and line["scaling"] == scaling
    ranks = line["ranks"]
    assert [r["rank"] for r in ranks] == [0, 1]
    assert ranks[0]["first"] + ranks[0]["streams"] == ranks[1]["first"]
    want = 65536 * (2 if scaling == "weak" else 1)
    assert line["streams_total"] == want == sum(r["streams"] for r in ranks)


def test_bench_under_torch_distributed_run():
    """The driver's launch: python -m torch.distributed.run --nproc-per-node 2
    --master-addr 127.0.0.1 bench.py --gpus 2 (ranks from the environment)."""
    line = _bench_line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                        "--dry-run", "--steps", "2"])
    assert line["n_gpus"] == 2 and line["world"] == 2 and line["streams_total"] == 131072
