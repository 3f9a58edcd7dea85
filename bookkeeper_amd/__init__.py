"""bookkeeper_amd — MI355X-native ledger-entry digest engine for Apache BookKeeper.

The product is the HIP/C-ABI library ``libbkdigest.so`` (include/bkdigest.h); this
package holds its sources (``csrc/``), the in-tree build and the host-side mirror of the
reference's checksum/digest provider surface (``checksum``: IntHash / Crc32cIntChecksum;
``digest``: DigestManager family).
"""
from ._native import CRC32, CRC32C, BkdError, NativeUnavailable  # noqa: F401

__all__ = ["CRC32", "CRC32C", "BkdError", "NativeUnavailable"]
