"""The slice of blb's internal/core + storageclass types the RS path touches.

Restated (not imported: the reference is Go) so the caller mirrors in tractserver.py /
client.py / curator.py read like the Go they follow.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass

TRACT_LENGTH = 8 * 1024 * 1024            # internal/core/constants.go:15
RS_CHUNK_VERSION = -317866832             # internal/core/constants.go:36
RS_PIECE_LENGTH = 64 * 1024 * 1024 - 64 * 1024 - 64   # internal/curator/storage_class_loop.go:22
MAX_RS_CHUNK_KEY = (1 << 48) - 1          # internal/core/ids.go (MaxRSChunkKey)
ENCODE_INCREMENT_PROD = 4 << 20           # internal/tractserver/config.go:117
ENCODE_INCREMENT_TEST = 1 << 20           # internal/tractserver/config.go:157


class Error(enum.Enum):
    """core.Error values used on the RS path (internal/core/errors.go)."""
    NoError = "no error"
    ErrVersionMismatch = "version mismatch"
    ErrShortRead = "short read"
    ErrCorruptData = "corrupt data"
    ErrEOF = "EOF"
    ErrInvalidArgument = "invalid argument"
    ErrHostNotExist = "host does not exist"
    ErrRPC = "rpc error"
    ErrUnknown = "unknown error"
    ErrAllocHost = "could not allocate host"
    ErrNoSuchTract = "tract does not exist"


class StorageClass(enum.IntEnum):
    """internal/core/StorageClass.go:7-13."""
    REPLICATED = 0
    RS_6_3 = 1
    RS_8_3 = 2
    RS_10_3 = 3
    RS_12_5 = 4


def rs_params(cls: StorageClass) -> tuple[int, int]:
    """storageclass.Class.RSParams (storageclass.go:37-46,142-144): parsed from RS_n_m."""
    if cls == StorageClass.REPLICATED:
        raise ValueError("REPLICATED has no RS params")
    _, n, m = cls.name.split("_")
    return int(n), int(m)


@dataclass(frozen=True)
class TractID:
    blob: int
    index: int

    def is_valid(self) -> bool:
        """internal/core/ids.go:237-239: a valid regular blob, or any RS-partition blob."""
        p = (self.blob >> 32) & 0xFFFFFFFF
        regular = (p & 0x3FFFFFFF) != 0 and (p >> 30) == 0 and (self.blob & 0xFFFFFFFF) > 0
        return regular or ((p & 0x3FFFFFFF) != 0 and (p >> 30) == 2)


def blob_id_from_parts(partition: int, key: int) -> int:
    """internal/core/ids.go:196-198 BlobIDFromParts."""
    return ((partition & 0xFFFFFFFF) << 32) | (key & 0xFFFFFFFF)


def tract_id_from_parts(blob: int, index: int) -> TractID:
    """internal/core/ids.go:242-244 TractIDFromParts."""
    return TractID(blob, index)


@dataclass(frozen=True)
class RSChunkID:
    """internal/core/ids.go:113 -- partition upper two bits 10 = RS partition."""
    partition: int
    id: int

    def is_valid(self) -> bool:
        p = self.partition & 0xFFFFFFFF
        return (p & 0x3FFFFFFF) != 0 and (p >> 30) == 2 and self.id != 0 and self.id <= MAX_RS_CHUNK_KEY

    def add(self, i: int) -> "RSChunkID":
        return RSChunkID(self.partition, self.id + i)

    def to_tract_id(self) -> TractID:
        return TractID(((self.partition & 0xFFFFFFFF) << 32) | ((self.id >> 16) & 0xFFFFFFFF),
                       self.id & 0xFFFF)


@dataclass(frozen=True)
class TSAddr:
    """core.TSAddr: a tractserver id and its host address."""
    id: int
    host: str
