"""Client side of the RS path on the MI355X engine: a restatement of blb's degraded read
(client/blb/client.go:1158-1190 readOneTractRS, client/blb/reconstruct.go:47-195
shouldReconstruct / reconstructOneTract) with the GPU Encoder's ReconstructData.

Kept from the Go code: the direct read first; reconstruction only when enabled, the class
is known and len(OtherHosts) == n+m; the target index is the entry whose TSID is ours
(else ErrInvalidArgument); requests go to every other non-empty host (fewer than n ->
ErrHostNotExist); the first n good replies win (short replies count as ErrShortRead); the
output lands in the caller's buffer thisB[0:length] and thisB[length:] is zero-padded;
a reconstruct failure -> ErrCorruptData; length < len(thisB) reports ErrEOF.
MaxInFlight bounds concurrent reconstructs with a semaphore (reconstruct.go:19,35-45).
"""
from __future__ import annotations

import threading
from concurrent.futures import ThreadPoolExecutor, as_completed
from dataclasses import dataclass, field
from typing import Optional, Protocol

import numpy as np

from . import reedsolomon, rpc
from .blbcore import RS_CHUNK_VERSION, Error, RSChunkID, StorageClass, TractID, rs_params


@dataclass
class TractPointer:
    """core.TractPointer (internal/core/messages.go:54-68)."""
    chunk: RSChunkID
    host: str
    tsid: int
    offset: int
    length: int
    cls: StorageClass = StorageClass.REPLICATED
    base_chunk: Optional[RSChunkID] = None
    other_hosts: list = field(default_factory=list)
    other_tsids: list = field(default_factory=list)


@dataclass
class TractResult:
    """client.go tractResult{len, read, err, badVersionHost}."""
    requested: int
    read: int
    err: Error


class TractserverReader(Protocol):
    def read(self, addr: str, tid: TractID, version: int, length: int, off: int
             ) -> tuple[Optional[np.ndarray], Error]: ...

    def read_into(self, addr: str, tid: TractID, version: int, b: np.ndarray, off: int
                  ) -> tuple[int, Error]: ...


@dataclass
class ReconstructBehavior:
    """reconstruct.go:24-28."""
    enabled: bool = True
    max_in_flight: int = 0


class Client:
    def __init__(self, tractservers: TractserverReader, behavior: ReconstructBehavior = ReconstructBehavior()):
        self.tractservers = tractservers
        self.behavior = behavior
        n = behavior.max_in_flight or 1  # defaultMaxReconstructInFlight
        self._sem = threading.Semaphore(n)
        self._pool = ThreadPoolExecutor(max_workers=32)
        self._encoders: dict = {}
        self._enc_lock = threading.Lock()
        self.reconstructs = 0

    def _encoder(self, n: int, m: int) -> reedsolomon.Encoder:
        # reconstruct.go:166 builds a fresh encoder per call; the GPU encoder caches its
        # device plans, so keep one per (n, m).
        with self._enc_lock:
            enc = self._encoders.get((n, m))
            if enc is None:
                enc = self._encoders[(n, m)] = reedsolomon.New(n, m)
            return enc

    # reconstruct.go:47-63
    def should_reconstruct(self, tract: TractPointer) -> bool:
        if not self.behavior.enabled:
            return False
        try:
            n, m = rs_params(StorageClass(tract.cls))
        except ValueError:
            return False
        return len(tract.other_hosts) == n + m

    # client.go:1158-1190
    def read_one_tract_rs(self, tract: TractPointer, thisB: np.ndarray, this_offset: int) -> TractResult:
        rs_tract = tract.chunk.to_tract_id()
        length = min(len(thisB), int(tract.length))
        offset = int(tract.offset) + this_offset
        read, err = self.tractservers.read_into(tract.host, rs_tract, RS_CHUNK_VERSION, thisB[:length], offset)
        if err not in (Error.NoError, Error.ErrEOF):
            if not self.should_reconstruct(tract):
                return TractResult(len(thisB), 0, err)
            return self.reconstruct_one_tract(tract, thisB, offset, length)
        thisB[read:] = 0  # pad with zeros (client.go:1193-1195)
        if int(tract.length) < len(thisB):
            err = Error.ErrEOF
        return TractResult(len(thisB), read, err)

    # reconstruct.go:65-195
    def reconstruct_one_tract(self, tract: TractPointer, thisB: np.ndarray, offset: int, length: int) -> TractResult:
        # reconstruct.go:126 `defer rpc.PutBuffer(p.res, true)` for each of the first n good
        # replies; errored replies and stragglers are dropped to the collector (rpc.py).
        kept: list = []
        try:
            with self._sem:
                return self._reconstruct(tract, thisB, offset, length, kept)
        finally:
            for b in kept:
                rpc.PutBuffer(b, True)

    def _reconstruct(self, tract: TractPointer, thisB: np.ndarray, offset: int, length: int,
                     kept: list) -> TractResult:
        n, m = rs_params(StorageClass(tract.cls))
        target, requests = -1, []
        for i, host in enumerate(tract.other_hosts):
            if tract.other_tsids[i] == tract.tsid:
                target = i
                continue
            if host == "":
                continue
            requests.append(i)
        if target < 0:
            return TractResult(len(thisB), 0, Error.ErrInvalidArgument)
        if len(requests) < n:
            return TractResult(len(thisB), 0, Error.ErrHostNotExist)

        def fetch(i):
            tid = tract.base_chunk.add(i).to_tract_id()
            res, err = self.tractservers.read(tract.other_hosts[i], tid, RS_CHUNK_VERSION, length, offset)
            if err in (Error.NoError, Error.ErrEOF) and (res is None or len(res) != length):
                err = Error.ErrShortRead
            return i, res, err

        data: list = [None] * (n + m)
        good, last_err = 0, Error.NoError
        futs = [self._pool.submit(fetch, i) for i in requests]
        for f in as_completed(futs):
            i, res, err = f.result()
            if err not in (Error.NoError, Error.ErrEOF):
                last_err = err
                continue
            good += 1
            data[i] = np.ascontiguousarray(res, dtype=np.uint8)
            kept.append(res)
            if good >= n:
                break
        # Go cancels the context here (reconstruct.go:154): reads not started yet are
        # dropped, running ones finish in the pool and their replies are ignored.
        for f in futs:
            f.cancel()
        if good < n:
            return TractResult(len(thisB), 0, last_err)
        try:
            enc = self._encoder(n, m)
        except reedsolomon.RSError:
            return TractResult(len(thisB), 0, Error.ErrInvalidArgument)
        # data[targetIdx] = thisB[0:0:length]: output lands in the caller's buffer.
        try:
            enc.ReconstructData(data, outs={target: thisB})
        except reedsolomon.RSError:
            return TractResult(len(thisB), 0, Error.ErrCorruptData)
        out = data[target]
        if out is None or len(out) != length or out.ctypes.data != thisB.ctypes.data:
            return TractResult(len(thisB), 0, Error.ErrCorruptData)
        thisB[length:] = 0
        self.reconstructs += 1
        return TractResult(len(thisB), length, Error.ErrEOF if length < len(thisB) else Error.NoError)
