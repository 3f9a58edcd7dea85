"""CPU: the composite-buffer leaf visit (ByteBufVisitor.java:72-191) over the buffer shapes of the
reference's CompositeByteBufUnwrapBugReproduceTest (bookkeeper-server/src/test/java/org/apache/
bookkeeper/proto/checksum/CompositeByteBufUnwrapBugReproduceTest.java:142-260): a composite with a
prefix and a reader index, two nested composites with empty components and duplicates, a sliced
composite. The visited leaves must concatenate to exactly the readable payload, in order, with no
empty leaf (the visitor skips them) — the property the digest chaining relies on."""
import numpy as np
import pytest

from bookkeeper_amd.bytebuf import CompositeBuffer

PREFIX = 7


def scenarios(payload: bytes):
    rng = np.random.default_rng(len(payload))
    prefix = rng.integers(0, 256, PREFIX, dtype=np.uint8).tobytes()
    plain = CompositeBuffer([payload])
    # wrapWithPrefixAndCompositeByteBufWithReaderIndexState (:215-228)
    prefixed = CompositeBuffer([prefix, payload])
    outer = CompositeBuffer([prefixed])
    outer.reader_index = PREFIX
    # ...MultipleCompositeByteBufWithReaderIndexStateAndMultipleLayersOfDuplicate (:231-250)
    inner = CompositeBuffer([CompositeBuffer([prefix, payload[:1000]]), payload[1000:], b""])
    outer2 = CompositeBuffer([inner, b""])
    outer2.reader_index = PREFIX
    dup = outer2.duplicate().duplicate()
    # wrapInCompositeByteBufAndSlice (:253-260)
    sliced = CompositeBuffer([prefix, bytearray(payload)]).slice(PREFIX, len(payload))
    return {"plain": plain, "reader_index": outer, "nested_duplicated": dup, "sliced": sliced}


@pytest.mark.parametrize("size", [16383, 16384])
def test_visit_concatenates_payload(size):
    payload = bytes(i & 0xFF for i in range(size))
    for name, buf in scenarios(payload).items():
        assert buf.readable_bytes() == size, name
        leaves = list(buf.visit(buf.reader_index, buf.readable_bytes()))
        assert all(n > 0 for _, _, n in leaves), name
        got = b"".join(bytes(memoryview(c).cast("B")[o:o + n]) for c, o, n in leaves)
        assert got == payload, name
        assert buf.readable() == payload, name


def test_visit_edges():
    b = CompositeBuffer([b"abc", b"", CompositeBuffer([b"de", b"f"])])
    assert b.capacity() == 6 and b.get_bytes(2, 3) == b"cde"
    assert list(b.visit(3, 0)) == []
    assert b.slice(1, 4).readable() == b"bcde"
    with pytest.raises(IndexError):
        list(b.visit(4, 3))
    with pytest.raises(IndexError):
        b.slice(5, 2)
