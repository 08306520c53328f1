"""Tractserver side of the RS path on the MI355X engine: a restatement of
Store.RSEncode / rsEncodeOne / reconstructAndVerify (internal/tractserver/store.go:1012-1144)
with the GPU Encoder from blb_amd.reedsolomon in place of klauspost's.

Behaviour kept from the Go code:
  * chunk-id range check -> ErrInvalidArgument; New() failure -> ErrInvalidArgument;
  * the piece is processed in EncodeIncrementSize windows (store.go:1028-1037);
  * each window: N concurrent CtlReads into data[indexMap[i]] (identity map when encoding),
    a short or failed read -> ErrVersionMismatch / the read's error; parity buffers come
    from an un-zeroed pool (rpc.GetBuffer); Encode, or Reconstruct + Verify
    (errVerifyFailed) when an indexMap is given; any coding error -> ErrUnknown;
    M concurrent CtlWrites of data[dataI] for dests with dataI >= 0 and ID != 0.

`pack_tracts` is Store.PackTracts (store.go:922-994): the packed
chunk is assembled on the GPU (blb_amd.pack.PackPieces) and kept HBM-resident in the
store's local chunk table, readable through `read` (the Store.Read slice the reference's
PackTracts test uses).

`pipeline=True` overlaps the reads of window i+1 with the writes of
window i, and the GPU coding of window i with the writes of window i-1.  Bytes written are
identical.  A failing read or coding step issues exactly the reference's calls; when a
CtlWrite of window i-1 fails, window i's reads have already been issued (no write of
window i is sent).
"""
from __future__ import annotations

import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Optional, Protocol, Sequence

import numpy as np

from . import pack, reedsolomon, rpc
from .hostcopy import to_numpy
from .blbcore import (ENCODE_INCREMENT_PROD, RS_CHUNK_VERSION, TRACT_LENGTH, Error, RSChunkID,
                      TractID, TSAddr)


class TractserverTalker(Protocol):
    """The two TractserverTalker calls rsEncodeOne makes (internal/tractserver/repl.go:26-32)."""

    def ctl_read(self, addr: str, tid: TractID, version: int, length: int, off: int
                 ) -> tuple[Optional[np.ndarray], Error]: ...

    def ctl_write(self, addr: str, tid: TractID, version: int, off: int, b: np.ndarray) -> Error: ...


class MemTractserverTalker:
    """Scripted talker, as store_test.go:21-81's memTractserverTalker: per-address FIFO of
    replies, every call recorded; an empty FIFO answers ErrRPC."""

    def __init__(self):
        self.lock = threading.Lock()
        self.ctl_read_calls: dict[str, list] = {}
        self.ctl_read_replies: dict[str, list] = {}
        self.ctl_write_calls: dict[str, list] = {}
        self.ctl_write_replies: dict[str, list] = {}

    def add_ctl_read_reply(self, addr: str, b: np.ndarray, err: Error) -> None:
        with self.lock:
            self.ctl_read_replies.setdefault(addr, []).append((np.array(b, dtype=np.uint8, copy=True), err))

    def add_ctl_write_reply(self, addr: str, err: Error) -> None:
        with self.lock:
            self.ctl_write_replies.setdefault(addr, []).append(err)

    def ctl_read(self, addr, tid, version, length, off):
        with self.lock:
            self.ctl_read_calls.setdefault(addr, []).append((tid, version, length, off))
            q = self.ctl_read_replies.get(addr) or []
            if not q:
                return None, Error.ErrRPC
            return q.pop(0)

    def ctl_write(self, addr, tid, version, off, b):
        with self.lock:
            self.ctl_write_calls.setdefault(addr, []).append((tid, version, np.array(b, copy=True), off))
            q = self.ctl_write_replies.get(addr) or []
            if not q:
                return Error.ErrRPC
            return q.pop(0)


class _VerifyFailed(Exception):
    """store.go:1144 errVerifyFailed."""


def reconstruct_and_verify(enc: reedsolomon.Encoder, data: list) -> None:
    """store.go:1132-1142: Reconstruct, then Verify (full parity recompute + compare); both
    run in one device round trip (blbrs_reconstruct_verify)."""
    if not enc.ReconstructAndVerify(data):
        raise _VerifyFailed("verification failed")


class Store:
    """The RS slice of internal/tractserver.Store."""

    def __init__(self, talker: TractserverTalker, encode_increment_size: int = ENCODE_INCREMENT_PROD,
                 pipeline: bool = False, batcher: Optional["reedsolomon.Batcher"] = None):
        self.tt = talker
        self.encode_increment_size = int(encode_increment_size)
        self.pipeline = pipeline
        # Shared by the Stores of one process (rsgpu.EnableBatching): the Encode / Reconstruct
        # / Verify calls of concurrent RSEncode RPCs share kernel launches.
        self.batcher = batcher
        self._pool = ThreadPoolExecutor(max_workers=32)
        self.local: dict[TractID, tuple] = {}   # tract id -> (device bytes, version)

    # ---- PackTracts (store.go:922-994) ----
    def pack_tracts(self, length: int, srcs: Sequence["pack.PackTractSpec"], dest: RSChunkID) -> Error:
        if not dest.is_valid() or not pack.check_tract_spec(srcs, length):
            return Error.ErrInvalidArgument
        dest_tract = dest.to_tract_id()
        self.local.pop(dest_tract, None)  # removeTract
        # Pull every source, sequentially, from the first replica that returns exactly
        # src.Length bytes (CtlRead of TractLength at offset 0, store.go:951-968).
        replies = []
        for src in srcs:
            for frm in src.from_:
                b, err = self.tt.ctl_read(frm.host, src.id, src.version, TRACT_LENGTH, 0)
                if err in (Error.NoError, Error.ErrEOF) and b is not None and len(b) == src.length:
                    replies.append(np.asarray(b, dtype=np.uint8))
                    break
            else:
                return Error.ErrRPC  # the half-written file is deleted: nothing is kept
        # The file ends at `length` when there are sources (pad, store.go:974-980), and is
        # empty otherwise.
        size = length if srcs else 0
        import torch
        piece = torch.empty((1, max(size, 1)), dtype=torch.uint8, device="cuda")
        if size:
            staged = torch.empty(max(sum(len(r) for r in replies), 1), dtype=torch.uint8).pin_memory()
            extents, pos = [], 0
            for src, r in zip(srcs, replies):
                staged[pos:pos + len(r)] = torch.from_numpy(r)
                extents.append((staged[pos:pos + len(r)], src.offset, src.length, 0))
                pos += len(r)
            pack.PackPieces(piece, size, extents)
            torch.cuda.current_stream().synchronize()  # `staged` is released on return
        self.local[dest_tract] = (piece[0, :size], RS_CHUNK_VERSION)
        return Error.NoError

    def read(self, tid: TractID, version: int, length: int, off: int):
        """Store.Read on the local chunk table: a short read is ErrEOF."""
        ent = self.local.get(tid)
        if ent is None:
            return None, Error.ErrNoSuchTract
        data, ver = ent
        if ver != version:
            return None, Error.ErrVersionMismatch
        b = to_numpy(data[off:off + length]) if off < data.numel() else np.zeros(0, np.uint8)
        return b, (Error.ErrEOF if len(b) < length else Error.NoError)

    # store.go:1014-1040
    def rs_encode(self, baseid: RSChunkID, length: int, srcs: Sequence[TSAddr], dests: Sequence[TSAddr],
                  index_map: Optional[Sequence[int]]) -> Error:
        N, M = len(srcs), len(dests)
        increment = self.encode_increment_size
        if not baseid.is_valid() or not baseid.add(N + M - 1).is_valid():
            return Error.ErrInvalidArgument
        try:
            enc = reedsolomon.New(N, M)
        except reedsolomon.RSError:
            return Error.ErrInvalidArgument
        if self.batcher is not None:
            enc.SetBatcher(self.batcher)
        windows = []
        off = 0
        while length > 0:
            ln = min(length, increment)
            windows.append((off, ln))
            length -= ln
            off += ln
        if not self.pipeline:
            for off, ln in windows:
                err = self._rs_encode_one(baseid, off, ln, srcs, dests, index_map, enc)
                if err != Error.NoError:
                    return err
            return Error.NoError
        return self._rs_encode_pipelined(baseid, windows, srcs, dests, index_map, enc)

    # ---- rsEncodeOne, split into its three stages (store.go:1042-1130) ----
    def _index_map(self, N, M, index_map):
        if not index_map:
            return list(range(N + M)), True
        if len(index_map) != N + M:
            return None, False
        return list(index_map), False

    def _gather(self, baseid, offset, length, srcs, imap, N, M):
        data: list = [None] * (N + M)

        def read(src_i, data_i):
            tid = baseid.add(data_i).to_tract_id()
            b, err = self.tt.ctl_read(srcs[src_i].host, tid, RS_CHUNK_VERSION, length, offset)
            if err not in (Error.NoError, Error.ErrEOF):
                return err
            if b is None or len(b) != length:
                return Error.ErrVersionMismatch
            data[data_i] = np.ascontiguousarray(b, dtype=np.uint8)
            return Error.NoError

        errs = list(self._pool.map(lambda a: read(*a), [(i, imap[i]) for i in range(N)]))
        for e in errs:
            if e != Error.NoError:
                return None, e
        return data, Error.NoError

    def _code(self, enc, data, encode, imap, N, length):
        try:
            if encode:
                for data_i in imap[N:]:
                    data[data_i] = rpc.GetBuffer(length)  # store.go:1099: not zeroed
                enc.Encode(data)
            else:
                reconstruct_and_verify(enc, data)
        except (reedsolomon.RSError, _VerifyFailed):
            return Error.ErrUnknown
        return Error.NoError

    def _scatter(self, baseid, offset, dests, imap, N, data):
        jobs = [(dest_i, data_i) for dest_i, data_i in enumerate(imap[N:])
                if data_i >= 0 and dests[dest_i].id != 0]

        def write(dest_i, data_i):
            tid = baseid.add(data_i).to_tract_id()
            return self.tt.ctl_write(dests[dest_i].host, tid, RS_CHUNK_VERSION, offset, data[data_i])

        errs = list(self._pool.map(lambda a: write(*a), jobs))
        for e in errs:
            if e != Error.NoError:
                return e
        return Error.NoError

    @staticmethod
    def _release(data):
        """store.go:1048-1052: `defer rpc.PutBuffer(b, true)` for everything in data."""
        for b in data or ():
            if b is not None:
                rpc.PutBuffer(b, True)

    def _scatter_release(self, baseid, offset, dests, imap, N, data):
        try:
            return self._scatter(baseid, offset, dests, imap, N, data)
        finally:
            self._release(data)

    def _rs_encode_one(self, baseid, offset, length, srcs, dests, index_map, enc) -> Error:
        N, M = len(srcs), len(dests)
        imap, encode = self._index_map(N, M, index_map)
        if imap is None:
            return Error.ErrInvalidArgument
        data, err = self._gather(baseid, offset, length, srcs, imap, N, M)
        if err != Error.NoError:
            return err
        try:
            err = self._code(enc, data, encode, imap, N, length)
            if err != Error.NoError:
                return err
            return self._scatter(baseid, offset, dests, imap, N, data)
        finally:
            self._release(data)

    def _rs_encode_pipelined(self, baseid, windows, srcs, dests, index_map, enc) -> Error:
        """Software pipeline over windows: gather(i+1) || scatter(i), code(i) || scatter(i-1)."""
        N, M = len(srcs), len(dests)
        imap, encode = self._index_map(N, M, index_map)
        if imap is None:
            return Error.ErrInvalidArgument
        stage = ThreadPoolExecutor(max_workers=2)
        try:
            nxt = stage.submit(self._gather, baseid, windows[0][0], windows[0][1], srcs, imap, N, M)
            pending_write = None
            for i, (off, ln) in enumerate(windows):
                data, err = nxt.result()
                if err != Error.NoError:
                    return err
                err = self._code(enc, data, encode, imap, N, ln)
                if err != Error.NoError:
                    self._release(data)
                    return err
                if pending_write is not None:
                    err = pending_write.result()
                    if err != Error.NoError:
                        return err
                # Window i+1's reads start only after window i is coded and window i-1's
                # writes succeeded (store.go:1029-1036 stops at the first failing window).
                if i + 1 < len(windows):
                    o2, l2 = windows[i + 1]
                    nxt = stage.submit(self._gather, baseid, o2, l2, srcs, imap, N, M)
                pending_write = stage.submit(self._scatter_release, baseid, off, dests, imap, N, data)
            return pending_write.result() if pending_write is not None else Error.NoError
        finally:
            stage.shutdown(wait=True)
