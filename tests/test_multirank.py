"""CPU rehearsal of the N>1 path with a world_size-2 gloo group (127.0.0.1).

The GPU path shards entries across ranks with no data-path collective. Here each
rank builds its shard of the global splitmix64 stream exactly as bench.py does
(shard_first_word), digests it with the oracle as a CPU stand-in for its GPU, and rank 0 checks
that the concatenated per-rank digests equal the digests of the unsharded batch; max_over_ranks
(the only collective bench.py uses) is checked too."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_per_rank, entry_len, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    import oracle
    from bench import max_over_ranks, shard_first_word
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fw = shard_first_word(rank, n_per_rank, entry_len)
        shard = oracle.fill_splitmix64(n_per_rank * entry_len, 42, fw)
        crcs = oracle.uniform(oracle.CRC32C, shard, entry_len, entry_len, n_per_rank)
        gathered = [torch.zeros(n_per_rank, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(crcs.astype(np.int64)))
        slowest = max_over_ranks(0.25 * (rank + 1))
        if rank == 0:
            q.put((np.concatenate([g.numpy() for g in gathered]).astype(np.uint32), slowest))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_digests_equal_unsharded(world):
    n_per_rank, entry_len = 512, 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_per_rank, entry_len, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, slowest = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    import oracle
    whole = oracle.fill_splitmix64(world * n_per_rank * entry_len, 42)
    want = oracle.uniform(oracle.CRC32C, whole, entry_len, entry_len, world * n_per_rank)
    assert (got == want).all()
    assert slowest == pytest.approx(0.25 * world)


def test_single_process_reduction_is_identity():
    from bench import max_over_ranks, shard_first_word
    assert max_over_ranks(1.5) == 1.5
    assert shard_first_word(3, 1 << 20, 4096) == 3 * (1 << 20) * 512


def test_bench_shard_parity_checker_cpu():
    """bench.py's N > 1 checker leg (shard_parity) on CPU tensors: a rank's correct digests match
    the oracle on the sampled entries (uniform and Zipf layouts), and one wrong sampled digest fails."""
    import torch

    import bench
    import oracle
    from bookkeeper_amd import checksum as ck
    n, L = 300, 256
    data = oracle.fill_splitmix64(n * L, 42)
    base = torch.from_numpy(data.copy())
    good = oracle.uniform(oracle.CRC32C, data, L, L, n)
    out = torch.from_numpy(good.view(np.int32).copy())
    assert bench.shard_parity(ck, torch, ck.CRC32C, "shard8m", base, out, n, L, None) == {"entries": n, "match": True}
    out[-1] ^= 1  # the sample always includes the last entry
    assert bench.shard_parity(ck, torch, ck.CRC32C, "shard8m", base, out, n, L, None)["match"] is False
    offs, lens = bench.zipf_index(200)
    zdata = oracle.fill_splitmix64(int(offs[-1] + lens[-1]), 7)
    zgood = oracle.batch(oracle.CRC32, zdata, offs, lens)
    zout = torch.from_numpy(zgood.view(np.int32).copy())
    chk = bench.shard_parity(ck, torch, ck.CRC32, "zipf", torch.from_numpy(zdata.copy()), zout, 200, 0, (offs, lens))
    assert chk == {"entries": 200, "match": True}


def _split_worker(rank, world, port, n, q):
    """One rank of config 3 split by bytes, as bench.py --config zipf_split does it: its entry range
    from byte_balanced_bounds, its span of the global stream generated from the span's first word,
    its index rebased to the span; digests by the oracle as the CPU stand-in for its GPU."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    import oracle
    from bench import zipf_index
    from bookkeeper_amd.shard import byte_balanced_bounds, shard_span
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        offs, lens = zipf_index(n)
        b = byte_balanced_bounds(lens, world)
        lo, hi = int(b[rank]), int(b[rank + 1])
        start, end = shard_span(offs, lens, lo, hi, align=128)
        span = oracle.fill_splitmix64(end - start, 42, start // 8)
        crcs = oracle.batch(oracle.CRC32C, span, offs[lo:hi] - start, lens[lo:hi])
        width = int(max(np.diff(b)))
        mine = torch.full((width,), -1, dtype=torch.int64)
        mine[:hi - lo] = torch.from_numpy(crcs.astype(np.int64))
        gathered = [torch.zeros(width, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, mine)
        if rank == 0:
            q.put((b, [g.numpy() for g in gathered]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_zipf_split_by_bytes_equals_unsplit(world):
    """config 3 over several ranks, contiguous entry ranges balanced by bytes; the
    ranks' digests, in rank order, are the unsplit batch's."""
    n = 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    b, parts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    import oracle
    from bench import zipf_index
    offs, lens = zipf_index(n)
    whole = oracle.fill_splitmix64(int(offs[-1] + lens[-1]), 42)
    want = oracle.batch(oracle.CRC32C, whole, offs, lens)
    got = np.concatenate([parts[r][:b[r + 1] - b[r]] for r in range(world)]).astype(np.uint32)
    assert got.size == n and (got == want).all()
    per = [int(lens[b[r]:b[r + 1]].sum()) for r in range(world)]
    assert max(per) <= lens.sum() / world + lens.max()
