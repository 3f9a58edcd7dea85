"""Materialises the inputs of tests/golden/crc_golden.json entries."""
import json
import os
import struct

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "crc_golden.json")


def load():
    return json.load(open(GOLDEN))


def load_4096():
    """The 4096-entry seeded set (lengths 0..70000, unaligned offsets into a 32 MiB stream)."""
    import numpy as np
    d = json.load(open(os.path.join(os.path.dirname(GOLDEN), "crc_golden_4096.json")))
    for k in ("offsets",):
        d[k] = np.array(d[k], dtype=np.uint64)
    for k in ("lengths", "seeds", "crc32c", "crc32"):
        d[k] = np.array(d[k], dtype=np.uint32)
    return d


def literal_bytes(v) -> bytes:
    if v.get("hex") is not None:
        return bytes.fromhex(v["hex"])
    if v.get("pattern") == "ramp":
        return bytes(i & 0xFF for i in range(v["len"]))
    if v.get("pattern") == "digest_frame":
        size = v["len"] - 32
        return struct.pack(">qqqq", 1, 1, 0, size) + bytes(i & 0xFF for i in range(size))
    raise ValueError(v["name"])
