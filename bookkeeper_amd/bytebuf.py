"""Composite buffers and the leaf visit DigestManager digests them with.

Reference: bookkeeper-server/src/main/java/org/apache/bookkeeper/util/ByteBufVisitor.java:72-191 walks
a (possibly nested, duplicated, sliced) Netty ``CompositeByteBuf`` down to its array / memory-address
leaves and hands each non-empty leaf range to a callback; ``DigestManager.update``
(proto/checksum/DigestManager.java:62-72, :380-392) chains ``internalUpdate(digest, leaf, off, len)``
over them, so the digest equals the digest of the concatenated bytes without copying them.

``CompositeBuffer`` is the host-side stand-in for those Netty buffers (components = bytes-like objects
or other composites; ``reader_index`` / ``writer_index`` / ``slice`` / ``duplicate`` as in Netty), and
``visit`` yields the same leaf ranges. On the device, entries made of several segments go through
``checksum.crc_batch_segments`` (``bkd_crc_batch_segments``) instead.
"""
from __future__ import annotations

from typing import Iterator, Sequence


def _leaf_len(c) -> int:
    return c.capacity() if isinstance(c, CompositeBuffer) else len(memoryview(c).cast("B"))


class CompositeBuffer:
    """Concatenation of components; Netty's absolute indexing (getBytes(index, ...)) over the whole
    content, with a readable window [reader_index, writer_index)."""

    def __init__(self, components: Sequence = (), reader_index: int = 0, writer_index: int | None = None):
        self._parts = []          # (component, start within the component, length)
        for c in components:
            self.add_component(c)
        self.reader_index = reader_index
        self.writer_index = self.capacity() if writer_index is None else writer_index

    @classmethod
    def _view(cls, parts, reader_index, writer_index) -> "CompositeBuffer":
        b = cls()
        b._parts = list(parts)
        b.reader_index, b.writer_index = reader_index, writer_index
        return b

    def add_component(self, c) -> "CompositeBuffer":
        """CompositeByteBuf.addComponent(true, c): appends c's readable bytes and extends the writer index."""
        if isinstance(c, CompositeBuffer):
            c = c.slice(c.reader_index, c.readable_bytes())
        n = _leaf_len(c)
        self._parts.append((c, 0, n))
        self.writer_index = self.capacity()
        return self

    def capacity(self) -> int:
        return sum(n for _, _, n in self._parts)

    def readable_bytes(self) -> int:
        return self.writer_index - self.reader_index

    def duplicate(self) -> "CompositeBuffer":
        """ByteBuf.duplicate(): shares the content, copies the indices."""
        return CompositeBuffer._view(self._parts, self.reader_index, self.writer_index)

    def slice(self, index: int, length: int) -> "CompositeBuffer":
        """ByteBuf.slice(index, length): a view of [index, index + length) with its own indices."""
        if index < 0 or length < 0 or index + length > self.capacity():
            raise IndexError("slice outside buffer")
        parts, pos = [], 0
        for c, s, n in self._parts:
            lo, hi = max(index, pos), min(index + length, pos + n)
            if lo < hi:
                parts.append((c, s + lo - pos, hi - lo))
            pos += n
        return CompositeBuffer._view(parts, 0, length)

    def visit(self, index: int, length: int) -> Iterator[tuple]:
        """ByteBufVisitor.visitBuffers(buf, index, length): the non-empty leaf ranges, in order, as
        (leaf bytes-like, offset, length); nested composites are descended."""
        if index < 0 or length < 0 or index + length > self.capacity():
            raise IndexError("range outside buffer")
        if length == 0:
            return
        pos = 0
        for c, s, n in self._parts:
            lo, hi = max(index, pos), min(index + length, pos + n)
            if lo < hi:
                if isinstance(c, CompositeBuffer):
                    yield from c.visit(s + lo - pos, hi - lo)
                else:
                    yield c, s + lo - pos, hi - lo
            pos += n

    def get_bytes(self, index: int, length: int) -> bytes:
        return b"".join(bytes(memoryview(c).cast("B")[o:o + n]) for c, o, n in self.visit(index, length))

    def readable(self) -> bytes:
        return self.get_bytes(self.reader_index, self.readable_bytes())
