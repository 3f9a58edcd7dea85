"""CPU: bench.py's host-side logic (no GPU): the workload chosen per GPU count, the shard layout of
config 4, and config 3's Zipf index."""
import numpy as np

import bench


def test_default_config_follows_gpu_count():
    # N = 1: BASELINE configs[1]; N > 1 (flag or torch.distributed.run's WORLD_SIZE): configs[3]'s shard
    assert bench.default_config(1, 1) == "uniform4k"
    for n in (2, 4, 8):
        assert bench.default_config(n, 1) == "shard8m"
        assert bench.default_config(1, n) == "shard8m"


def test_config4_shards_tile_the_global_stream():
    per, L = 8 << 20, 4096
    firsts = [bench.shard_first_word(r, per, L) for r in range(8)]
    assert firsts[0] == 0
    # consecutive shards are adjacent slices of one stream: 64M x 4 KiB in 8-byte words
    assert all(b - a == per * L // 8 for a, b in zip(firsts, firsts[1:]))
    assert firsts[-1] + per * L // 8 == (64 << 20) * L // 8


def test_zipf_index_matches_survey_shape():
    offs, lens = bench.zipf_index(1 << 16)
    assert lens.min() >= 64 and lens.max() <= 65536
    assert (offs[1:] == offs[:-1] + lens[:-1]).all()  # packed back to back
    assert 5000 < lens.mean() < 8000  # mean ~6 484 B on 1M entries
    o2, l2 = bench.zipf_index(1 << 16)
    assert np.array_equal(offs, o2) and np.array_equal(lens, l2)  # seeded


def test_only_config2_carries_the_headline_metric():
    """BASELINE.json's metric names config 2 (1M x 4 KiB, CRC32C) only; every other
    workload's line names itself (Zipf, CRC32, config 4's shard), so none can be read as the headline."""
    import json
    import os
    base = json.load(open(os.path.join(os.path.dirname(bench.__file__), "BASELINE.json")))
    assert bench.metric_for("uniform4k", "crc32c") == base["metric"] == bench.METRIC
    others = [bench.metric_for(c, a) for c in ("uniform4k", "shard8m", "zipf", "zipf_split", "indexed4k")
              for a in ("crc32c", "crc32")
              if (c, a) != ("uniform4k", "crc32c")]
    assert len(set(others)) == len(others) and base["metric"] not in others
    assert "Zipf" in bench.metric_for("zipf", "crc32") and "CRC32 " in bench.metric_for("zipf", "crc32")
    assert "config 4" in bench.metric_for("shard8m", "crc32c")
    assert "split across the GPUs by bytes" in bench.metric_for("zipf_split", "crc32c")
