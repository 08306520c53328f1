"""Host-side mirror of github.com/klauspost/reedsolomon's Encoder (the interface blb binds),
running on the MI355X engine through the C ABI in include/blb_rs.h.

Same names, argument meaning and error behaviour as the Go library at the pinned version
(/root/reference/go.mod:20), so that the parity tests read like blb's own tests:

    enc = reedsolomon.New(n, m)          # internal/tractserver/store.go:1022
    enc.Encode(shards)                   # store.go:1099
    enc.Reconstruct(shards)              # store.go:1133   (reconstructAndVerify)
    ok = enc.Verify(shards)              # store.go:1136
    enc.ReconstructData(shards)          # client/blb/reconstruct.go:173

`shards` is a list of k+m shards, data first.  A shard is a 1-D C-contiguous numpy uint8
array (host memory: copied through the GPU) or a 1-D torch.uint8 CUDA tensor (device
memory: coded in place on the current torch stream).  For Reconstruct*, a missing shard
is None or empty; like klauspost's `make`, a fresh buffer is allocated and stored back into
the list, unless `outs={index: buffer}` supplies one (klauspost reuses cap >= size --
the client's `thisB[0:0:length]` trick at client/blb/reconstruct.go:172-175).

Batched device-resident methods (EncodeBatch / ReconstructBatch / VerifyBatch) take a
torch.uint8 CUDA tensor [B, k+m, S] of stripes -- the bench / batched-caller path.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib


class RSError(Exception):
    """Base of the klauspost error values."""
    code = 0


class ErrInvShardNum(RSError):
    code = -1


class ErrMaxShardNum(RSError):
    code = -2


class ErrTooFewShards(RSError):
    code = -3


class ErrShardNoData(RSError):
    code = -4


class ErrShardSize(RSError):
    code = -5


class ErrSingular(RSError):
    code = -6


class ErrInvalidArgument(RSError):
    code = -7


class ErrHIP(RSError):
    code = -8


class ErrNoDevice(RSError):
    code = -9


class ErrLimit(RSError):
    """The pinned-memory live limit is reached (blbrs_pool_set_live_limit): use pageable memory."""
    code = -10


_ERRORS = {c.code: c for c in (ErrInvShardNum, ErrMaxShardNum, ErrTooFewShards, ErrShardNoData,
                                ErrShardSize, ErrSingular, ErrInvalidArgument, ErrHIP, ErrNoDevice, ErrLimit)}


def _check(rc: int) -> None:
    if rc != 0:
        lib = _lib.load()
        msg = lib.blbrs_last_error().decode() or lib.blbrs_strerror(rc).decode()
        raise _ERRORS.get(rc, RSError)(msg)


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _torch_stream(dev_tensor) -> int:
    import torch
    return torch.cuda.current_stream(dev_tensor.device).cuda_stream


def _shard_len(s) -> int:
    if s is None:
        return 0
    return int(s.numel()) if _is_torch(s) else int(s.size)


def _host_ptr(a: np.ndarray) -> int:
    if not isinstance(a, np.ndarray) or a.dtype != np.uint8 or a.ndim != 1 or not a.flags.c_contiguous:
        raise ErrInvalidArgument("host shards must be 1-D C-contiguous numpy uint8 arrays")
    return a.ctypes.data


def _dev_ptr(t) -> int:
    import torch
    if t.dtype != torch.uint8 or t.dim() != 1 or not t.is_cuda or (t.numel() > 1 and t.stride(0) != 1):
        raise ErrInvalidArgument("device shards must be 1-D contiguous torch.uint8 CUDA tensors")
    return t.data_ptr()


class Encoder:
    """reedsolomon.Encoder for (DataShards, ParityShards), backed by libblbrs."""

    def __init__(self, data_shards: int, parity_shards: int, devices: Optional[Sequence[int]] = None):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        if devices is None:
            _check(self._lib.blbrs_new(int(data_shards), int(parity_shards), ctypes.byref(h)))
        else:
            devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
            _check(self._lib.blbrs_new_on(int(data_shards), int(parity_shards), devs, len(devices), ctypes.byref(h)))
        self._h = h
        self.DataShards = int(data_shards)
        self.ParityShards = int(parity_shards)
        self.Shards = self.DataShards + self.ParityShards

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.blbrs_free(h)
            self._h = None

    def SetBatcher(self, batcher: Optional["Batcher"]) -> None:
        """Route this encoder's host Encode / Verify / Reconstruct / ReconstructData /
        ReconstructAndVerify calls through `batcher` (None detaches).  Results and errors are
        unchanged; concurrent callers share launches."""
        _check(self._lib.blbrs_encoder_set_batcher(self._h, batcher._h if batcher else None))
        self._batcher = batcher  # keep it alive while attached

    # ---- introspection ----
    def Devices(self) -> list:
        """The encoder's device list (host calls run on its least-loaded entry)."""
        n = ctypes.c_int(0)
        _check(self._lib.blbrs_encoder_devices(self._h, None, 0, ctypes.byref(n)))
        out = (ctypes.c_int * max(1, n.value))()
        _check(self._lib.blbrs_encoder_devices(self._h, out, n.value, ctypes.byref(n)))
        return list(out[:n.value])

    def LaneStats(self, lane: int) -> dict:
        """Load of entry `lane` of the device list: calls / shard bytes routed to it so far and
        in flight now (blbrs_encoder_lane_stats)."""
        st = _lib.LaneStats()
        _check(self._lib.blbrs_encoder_lane_stats(self._h, int(lane), ctypes.byref(st)))
        return {f: int(getattr(st, f)) for f, _ in st._fields_}

    def matrix(self) -> np.ndarray:
        out = np.zeros((self.Shards, self.DataShards), dtype=np.uint8)
        _check(self._lib.blbrs_matrix(self._h, out.ctypes.data, out.size))
        return out

    def compiled_network(self) -> dict:
        """Which kernels run this encoder's Encode as a bit-plane XOR network rather than the
        v_perm tables (blbrs_encoder_compiled_network): code (rs_code_kernel: Encode / Verify),
        tile (fused encode+CRC), pack (PackTracts + Encode), rtc (a network compiled at run
        time for k outside the library's compiled list)."""
        bits = int(self._lib.blbrs_encoder_compiled_network(self._h))
        return {"code": bool(bits & 1), "tile": bool(bits & 2), "pack": bool(bits & 4), "rtc": bool(bits & 8)}

    # ---- helpers ----
    def _arrays(self, shards, n):
        ptrs = (ctypes.c_void_p * n)()
        lens = (ctypes.c_size_t * n)()
        return ptrs, lens

    def _kind(self, shards) -> Optional[str]:
        kinds = {("dev" if _is_torch(s) else "host") for s in shards if _shard_len(s)}
        if len(kinds) > 1:
            raise ErrInvalidArgument("mixing host and device shards in one call")
        return kinds.pop() if kinds else None

    @staticmethod
    def _check_sizes(lens: Sequence[int], nilok: bool) -> int:
        """reedsolomon.go checkShards / shardSize."""
        size = next((x for x in lens if x), 0)
        if size == 0:
            raise ErrShardNoData("no shard data")
        for x in lens:
            if x != size and (x != 0 or not nilok):
                raise ErrShardSize("shard sizes do not match")
        return size

    # ---- Encoder interface ----
    def Encode(self, shards: list) -> None:
        """Encode parity for shards[0:k] into shards[k:k+m] (fully overwritten)."""
        n = self.Shards
        if len(shards) != n:
            raise ErrTooFewShards("too few shards given")
        lens = [_shard_len(s) for s in shards]
        self._check_sizes(lens, nilok=False)
        if self._kind(shards) == "dev":
            ptrs = (ctypes.c_void_p * n)(*[_dev_ptr(s) for s in shards])
            _check(self._lib.blbrs_encode_dev_ptrs(self._h, ptrs, 1, lens[0], _torch_stream(shards[0])))
            return
        ptrs = (ctypes.c_void_p * n)(*[_host_ptr(s) for s in shards])
        L = (ctypes.c_size_t * n)(*lens)
        _check(self._lib.blbrs_encode(self._h, ptrs, L))

    def Verify(self, shards: list) -> bool:
        """True when the parity shards equal the encoding of the data shards."""
        n = self.Shards
        if len(shards) != n:
            raise ErrTooFewShards("too few shards given")
        lens = [_shard_len(s) for s in shards]
        self._check_sizes(lens, nilok=False)
        if self._kind(shards) == "dev":
            import torch
            flag = torch.empty(1, dtype=torch.int32, device=shards[0].device)
            ptrs = (ctypes.c_void_p * n)(*[_dev_ptr(s) for s in shards])
            _check(self._lib.blbrs_verify_dev_ptrs(self._h, ptrs, 1, lens[0], flag.data_ptr(),
                                                    _torch_stream(shards[0])))
            return int(flag.item()) == 0
        ptrs = (ctypes.c_void_p * n)(*[_host_ptr(s) for s in shards])
        L = (ctypes.c_size_t * n)(*lens)
        ok = ctypes.c_int(0)
        _check(self._lib.blbrs_verify(self._h, ptrs, L, ctypes.byref(ok)))
        return bool(ok.value)

    def _reconstruct(self, shards: list, data_only: bool, outs: Optional[dict], verify: bool = False):
        n = self.Shards
        if len(shards) != n:
            raise ErrTooFewShards("too few shards given")
        lens = [_shard_len(s) for s in shards]
        size = self._check_sizes(lens, nilok=True)
        present = [x != 0 for x in lens]
        if all(present):
            return self.Verify(shards) if verify else None
        if sum(present) < self.DataShards:
            raise ErrTooFewShards("too few shards given")
        kind = self._kind(shards)
        outs = outs or {}
        produce = [i for i in range(n) if not present[i] and (i < self.DataShards or not data_only)]
        bufs = list(shards)
        for i in produce:
            if i in outs:
                o = outs[i]
                if _shard_len(o) < size:
                    raise ErrInvalidArgument(f"output buffer for shard {i} is smaller than the shard size")
                bufs[i] = o[:size]
            elif kind == "dev":
                import torch
                ref = next(s for s in shards if _shard_len(s))
                bufs[i] = torch.empty(size, dtype=torch.uint8, device=ref.device)
            else:
                bufs[i] = np.empty(size, dtype=np.uint8)
        if kind == "dev":
            ptrs = (ctypes.c_void_p * n)(*[_dev_ptr(bufs[i]) if (present[i] or i in produce) else None
                                           for i in range(n)])
            pres = (ctypes.c_uint8 * n)(*[1 if p else 0 for p in present])
            ref = next(s for s in shards if _shard_len(s))
            _check(self._lib.blbrs_reconstruct_dev_ptrs(self._h, ptrs, 1, size, pres, int(data_only),
                                                         _torch_stream(ref)))
            for i in produce:
                shards[i] = bufs[i]
            return self.Verify(shards) if verify else None
        ptrs = (ctypes.c_void_p * n)(*[_host_ptr(bufs[i]) if (present[i] or i in produce) else None
                                       for i in range(n)])
        L = (ctypes.c_size_t * n)(*lens)
        ok = None
        if verify:
            okc = ctypes.c_int(0)
            _check(self._lib.blbrs_reconstruct_verify(self._h, ptrs, L, ctypes.byref(okc)))
            ok = bool(okc.value)
        else:
            fn = self._lib.blbrs_reconstruct_data if data_only else self._lib.blbrs_reconstruct
            _check(fn(self._h, ptrs, L))
        for i in produce:
            shards[i] = bufs[i]
        return ok

    def Reconstruct(self, shards: list, outs: Optional[dict] = None) -> None:
        """Rebuild every missing shard (data and parity) in the list."""
        self._reconstruct(shards, False, outs)

    def ReconstructData(self, shards: list, outs: Optional[dict] = None) -> None:
        """Rebuild missing data shards only; parity slots stay missing."""
        self._reconstruct(shards, True, outs)

    def ReconstructAndVerify(self, shards: list, outs: Optional[dict] = None) -> bool:
        """reconstructAndVerify (internal/tractserver/store.go:1132-1142): Reconstruct, then
        Verify the completed stripe -- for host shards in one device round trip."""
        return bool(self._reconstruct(shards, False, outs, verify=True))

    # ---- batched device-resident path ----
    def _stripes(self, stripes):
        import torch
        if not (_is_torch(stripes) and stripes.is_cuda and stripes.dtype == torch.uint8 and stripes.dim() == 3):
            raise ErrInvalidArgument("stripes must be a [B, k+m, S] torch.uint8 CUDA tensor")
        B, n, S = stripes.shape
        if n != self.Shards:
            raise ErrTooFewShards("too few shards given")
        if S > 1 and stripes.stride(2) != 1:
            raise ErrInvalidArgument("shard bytes must be contiguous (stride(2) == 1)")
        return B, S, stripes.stride(1), stripes.stride(0)

    def EncodeBatch(self, stripes, stream: Optional[int] = None) -> None:
        """Encode every stripe of a [B, k+m, S] device tensor in place (async on the stream)."""
        B, S, ss, bs = self._stripes(stripes)
        st = _torch_stream(stripes) if stream is None else stream
        _check(self._lib.blbrs_encode_dev(self._h, stripes.data_ptr(), ss, bs, B, S, st))

    def EncodeBatchCRC(self, stripes, block: int = 0, stream: Optional[int] = None, phase: int = 0,
                       seeds=None):
        """EncodeBatch fused with the CRC-32C of the parity it writes (one HBM pass).

        Returns a [m, B, nblocks] torch.int32 CUDA tensor (the uint32 CRCs' bit patterns):
        entry [j, b, i] = crc32.Checksum(block i of parity shard k+j of stripe b).
        block = 0: one block per shard (the bulk RPC frame CRC, pkg/rpc/bulk_codec.go:47);
        65532 = ChecksumFile blocks (pkg/disk/checksum_block.go:18-34).

        phase / seeds (blbrs_encode_crc_dev_at): the shards are a window of the parity piece
        whose byte 0 sits `phase` bytes into a block (rsEncodeOne's window at offset 4 MiB*i:
        phase = 4 MiB*i mod 65532); nblocks = ceil((phase + S) / block) and entry [j, b, 0]
        continues seeds[j, b] (crc32.Update).  seeds: [m, B] int32 CUDA tensor or None."""
        import torch
        B, S, ss, bs = self._stripes(stripes)
        if block <= 0:
            blk, phase = S, 0
        else:
            blk = block
        nblocks = (S + phase + blk - 1) // blk if S else 0
        out = torch.empty((self.ParityShards, B, nblocks), dtype=torch.int32, device=stripes.device)
        st = _torch_stream(stripes) if stream is None else stream
        sp = None
        if seeds is not None:
            if not (_is_torch(seeds) and seeds.dtype == torch.int32 and seeds.is_contiguous()
                    and tuple(seeds.shape) == (self.ParityShards, B) and seeds.device == stripes.device):
                raise ErrInvalidArgument("seeds must be a contiguous [m, B] int32 tensor on the stripes' device")
            sp = seeds.data_ptr()
        _check(self._lib.blbrs_encode_crc_dev_at(self._h, stripes.data_ptr(), ss, bs, B, S, blk, phase, sp,
                                                 out.data_ptr(), st))
        return out

    def ReconstructBatch(self, stripes, present: Sequence[bool], data_only: bool = False,
                         stream: Optional[int] = None) -> None:
        """Rebuild the shards marked absent in `present` for every stripe, in place."""
        B, S, ss, bs = self._stripes(stripes)
        if len(present) != self.Shards:
            raise ErrTooFewShards("too few shards given")
        pres = (ctypes.c_uint8 * self.Shards)(*[1 if p else 0 for p in present])
        st = _torch_stream(stripes) if stream is None else stream
        _check(self._lib.blbrs_reconstruct_dev(self._h, stripes.data_ptr(), ss, bs, B, S, pres,
                                               int(data_only), st))

    def ReconstructBatchCRC(self, stripes, present: Sequence[bool], block: int = 0, data_only: bool = False,
                            stream: Optional[int] = None, phase: int = 0, seeds=None):
        """ReconstructBatch fused with the CRC-32C of every rebuilt shard (the recovery RPC's
        CtlWrite of the rebuilt pieces, store.go:1110-1120).  Returns [r, B, nblocks] int32
        (r = rebuilt shards: missing data ascending, then missing parity unless data_only), or
        None when nothing is rebuilt.  block / phase / seeds ([r, B] int32) as EncodeBatchCRC."""
        import torch
        B, S, ss, bs = self._stripes(stripes)
        if len(present) != self.Shards:
            raise ErrTooFewShards("too few shards given")
        rows = [i for i in range(self.Shards) if not present[i] and (i < self.DataShards or not data_only)]
        if not rows:
            return None
        if block <= 0:
            blk, phase = S, 0
        else:
            blk = block
        nblocks = (S + phase + blk - 1) // blk if S else 0
        out = torch.empty((len(rows), B, nblocks), dtype=torch.int32, device=stripes.device)
        sp = None
        if seeds is not None:
            if not (_is_torch(seeds) and seeds.dtype == torch.int32 and seeds.is_contiguous()
                    and tuple(seeds.shape) == (len(rows), B) and seeds.device == stripes.device):
                raise ErrInvalidArgument("seeds must be a contiguous [r, B] int32 tensor on the stripes' device")
            sp = seeds.data_ptr()
        pres = (ctypes.c_uint8 * self.Shards)(*[1 if p else 0 for p in present])
        st = _torch_stream(stripes) if stream is None else stream
        _check(self._lib.blbrs_reconstruct_crc_dev_at(self._h, stripes.data_ptr(), ss, bs, B, S, pres,
                                                      int(data_only), blk, phase, sp, out.data_ptr(), st))
        return out

    def ReconstructAndVerifyBatch(self, stripes, present: Sequence[bool], stream: Optional[int] = None):
        """reconstructAndVerify (store.go:1132-1142) on a device batch in one pass: the shards
        marked absent are rebuilt in place; returns a [B] torch.bool CUDA tensor, True where
        the completed stripe verifies."""
        import torch
        B, S, ss, bs = self._stripes(stripes)
        if len(present) != self.Shards:
            raise ErrTooFewShards("too few shards given")
        flags = torch.empty(B, dtype=torch.int32, device=stripes.device)
        pres = (ctypes.c_uint8 * self.Shards)(*[1 if p else 0 for p in present])
        st = _torch_stream(stripes) if stream is None else stream
        _check(self._lib.blbrs_reconstruct_verify_dev(self._h, stripes.data_ptr(), ss, bs, B, S, pres,
                                                      flags.data_ptr(), st))
        return flags == 0

    def VerifyBatch(self, stripes, stream: Optional[int] = None):
        """Returns a [B] torch.bool CUDA tensor: True where the stripe's parity is consistent."""
        import torch
        B, S, ss, bs = self._stripes(stripes)
        flags = torch.empty(B, dtype=torch.int32, device=stripes.device)
        st = _torch_stream(stripes) if stream is None else stream
        _check(self._lib.blbrs_verify_dev(self._h, stripes.data_ptr(), ss, bs, B, S, flags.data_ptr(), st))
        return flags == 0

    # ---- multi-device parts (one [B_p, k+m, S] CUDA tensor per device share) ----
    def _parts(self, parts):
        arr = (_lib.DevPart * len(parts))()
        S = None
        for i, t in enumerate(parts):
            B, s_, ss, bs = self._stripes(t)
            if S is None:
                S = s_
            elif s_ != S:
                raise ErrShardSize("shard sizes do not match")
            arr[i] = _lib.DevPart(t.data_ptr(), ss, bs, B, _torch_stream(t))
        return arr, (S or 0)

    def EncodeParts(self, parts: Sequence) -> None:
        """Encode every part in place, each on its own device and current torch stream."""
        arr, S = self._parts(parts)
        _check(self._lib.blbrs_encode_parts(self._h, arr, len(parts), S))

    def ReconstructParts(self, parts: Sequence, present: Sequence[bool], data_only: bool = False) -> None:
        if len(present) != self.Shards:
            raise ErrTooFewShards("too few shards given")
        arr, S = self._parts(parts)
        pres = (ctypes.c_uint8 * self.Shards)(*[1 if p else 0 for p in present])
        _check(self._lib.blbrs_reconstruct_parts(self._h, arr, len(parts), S, pres, int(data_only)))

    def VerifyParts(self, parts: Sequence) -> list:
        """[B_p] torch.bool per part: True where the stripe's parity is consistent."""
        import torch
        arr, S = self._parts(parts)
        flags = [torch.empty(t.shape[0], dtype=torch.int32, device=t.device) for t in parts]
        fp = (ctypes.c_void_p * len(parts))(*[f.data_ptr() for f in flags])
        _check(self._lib.blbrs_verify_parts(self._h, arr, len(parts), S, fp))
        return [f == 0 for f in flags]

    def EncodeHostBatch(self, stripes: Sequence[Sequence[np.ndarray]], nstreams: int = 0) -> None:
        """Streaming encode of host-resident stripes (blbrs_encode_host_batch).  nstreams = 0:
        pinned stripes coded in place over PCIe (zero copy), pageable ones staged by CPU copies;
        nstreams >= 1: pinned stripes through the copy engines (hipMemcpyAsync H2D, kernel on a
        device ring, D2H) on that many streams."""
        n = self.Shards
        B = len(stripes)
        if B == 0:
            return
        S = _shard_len(stripes[0][0])
        flat = []
        for st in stripes:
            if len(st) != n:
                raise ErrTooFewShards("too few shards given")
            for s in st:
                if _shard_len(s) != S:
                    raise ErrShardSize("shard sizes do not match")
                flat.append(_host_ptr(s))
        ptrs = (ctypes.c_void_p * len(flat))(*flat)
        _check(self._lib.blbrs_encode_host_batch(self._h, ptrs, B, S, int(nstreams)))


class Batcher:
    """Batching queue for concurrent host Encode / Verify / Reconstruct / ReconstructData calls
    (client/blb/reconstruct.go:65-195 with MaxInFlight > 1, and
    the tractserver's concurrent RSEncode RPCs, store.go:1099).  Calls that arrive within
    `window_us` of the first waiting one (or until `max_batch` wait) run as one kernel launch
    per (shape, plan, length) group.  window_us = 0 (default) batches naturally: a free lane
    takes whatever is queued at once, and calls that arrive while the lanes are busy form
    the next batch, so a lone caller waits for nothing.  Attach with
    Encoder.SetBatcher; free only after detaching from every encoder."""

    def __init__(self, max_batch: int = 64, window_us: int = 0, devices: Optional[Sequence[int]] = None):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        if devices is None:
            _check(self._lib.blbrs_batcher_new(int(max_batch), int(window_us), ctypes.byref(h)))
        else:
            devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
            _check(self._lib.blbrs_batcher_new_on(int(max_batch), int(window_us), devs, len(devices),
                                                  ctypes.byref(h)))
        self._h = h

    def stats(self) -> tuple[int, int]:
        """(calls served, kernel launches issued)."""
        r, l = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._lib.blbrs_batcher_stats(self._h, ctypes.byref(r), ctypes.byref(l)))
        return int(r.value), int(l.value)

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.blbrs_batcher_free(h)
            self._h = None

    def __del__(self):
        self.close()


def New(data_shards: int, parity_shards: int, devices: Optional[Sequence[int]] = None) -> Encoder:
    """reedsolomon.New(dataShards, parityShards) -> Encoder (raises ErrInvShardNum /
    ErrMaxShardNum like the Go constructor).  `devices`: the device list host calls spread
    over (blbrs_new_on); default = the process default list (every visible device)."""
    return Encoder(data_shards, parity_shards, devices)


def set_default_devices(devices: Optional[Sequence[int]]) -> None:
    devs = list(devices or [])
    arr = (ctypes.c_int * max(1, len(devs)))(*devs)
    _check(_lib.load().blbrs_set_default_devices(arr if devs else None, len(devs)))


# ---- pinned buffer pool: rpc.GetBuffer / PutBuffer (pkg/rpc/pool.go:16-62) ----

def GetBuffer(n: int) -> np.ndarray:
    """A length-n uint8 array in pooled pinned memory (NOT zeroed; capacity class of blb's
    pool).  Host-memory calls on such shards run zero-copy.  Give it back with PutBuffer and
    do not touch it afterwards."""
    lib = _lib.load()
    p = ctypes.c_void_p()
    cap = ctypes.c_size_t(0)
    _check(lib.blbrs_buffer_get(int(n), ctypes.byref(p), ctypes.byref(cap)))
    return np.ctypeslib.as_array((ctypes.c_uint8 * int(n)).from_address(p.value))


def PutBuffer(buf: np.ndarray) -> None:
    _check(_lib.load().blbrs_buffer_put(buf.__array_interface__["data"][0]))


def set_live_limit(nbytes: int) -> None:
    """Cap on pinned bytes alive at once: buffers handed out by GetBuffer plus memory
    registered by rpc.GetBuffer's pools (0 = no cap; default 16 GiB)."""
    _check(_lib.load().blbrs_pool_set_live_limit(int(nbytes)))


def pool_stats() -> dict:
    st = _lib.PoolStats()
    _check(_lib.load().blbrs_get_pool_stats(ctypes.byref(st)))
    return {f: int(getattr(st, f)) for f, _ in st._fields_}


def device_stats(device: int) -> dict:
    st = _lib.DeviceStats()
    _check(_lib.load().blbrs_get_device_stats(int(device), ctypes.byref(st)))
    return {f: int(getattr(st, f)) for f, _ in st._fields_}


def set_worker_limit(per_device: int) -> None:
    _check(_lib.load().blbrs_set_worker_limit(int(per_device)))


def trim() -> None:
    _check(_lib.load().blbrs_trim())


def plan_stats() -> dict:
    """Plans built since the process started (blbrs_plan_stats): host (inversions) and device
    (table uploads)."""
    h, d = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _check(_lib.load().blbrs_plan_stats(ctypes.byref(h), ctypes.byref(d)))
    return {"host_plans": h.value, "device_plans": d.value}


def set_device(device: int) -> None:
    _check(_lib.load().blbrs_set_device(int(device)))


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(_lib.load().blbrs_device_count(ctypes.byref(n)))
    return n.value


# ---- NUMA placement (include/blb_rs.h) ----

def device_numa_node(device: int) -> int:
    n = ctypes.c_int(-1)
    _check(_lib.load().blbrs_device_numa_node(int(device), ctypes.byref(n)))
    return int(n.value)


def set_device_numa_node(device: int, node: int) -> None:
    _check(_lib.load().blbrs_set_device_numa_node(int(device), int(node)))


def host_numa_node(buf) -> int:
    """Node recorded for the pool / registered buffer holding `buf` (numpy array or address)."""
    addr = buf if isinstance(buf, int) else buf.__array_interface__["data"][0]
    n = ctypes.c_int(-1)
    _check(_lib.load().blbrs_host_numa_node(ctypes.c_void_p(addr), ctypes.byref(n)))
    return int(n.value)


def lane_policy(nodes: Sequence[int], loads: Sequence[int], start: int, node: int) -> int:
    """The library's lane pick (runtime pick_lane_policy) over explicit lanes."""
    n = len(nodes)
    na = (ctypes.c_int * n)(*nodes)
    la = (ctypes.c_int64 * n)(*loads)
    out = ctypes.c_size_t(0)
    _check(_lib.load().blbrs_lane_policy(na, la, n, int(start), int(node), ctypes.byref(out)))
    return int(out.value)


# ---- A/B knobs and run-time decode networks (include/blb_rs.h) ----

def set_tuning(name: str, value: int) -> None:
    """Set a library knob (BLBRS_BITSLICE, BLBRS_RTC, ...; read from the environment once, at
    load, and changed only through this call)."""
    _check(_lib.load().blbrs_set_tuning(name.encode(), int(value)))


def get_tuning(name: str) -> int:
    v = ctypes.c_long(0)
    _check(_lib.load().blbrs_get_tuning(name.encode(), ctypes.byref(v)))
    return int(v.value)


class tuning:
    """Context manager: `with rs.tuning(BLBRS_BITSLICE=0): ...` sets knobs and restores them."""

    def __init__(self, **knobs):
        self._knobs = knobs
        self._old = {}

    def __enter__(self):
        for k, v in self._knobs.items():
            self._old[k] = get_tuning(k)
            set_tuning(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self._old.items():
            set_tuning(k, v)
        return False


_KNOB_START = {}


def use_knobs(env: dict) -> None:
    """A/B drivers: set exactly the knobs in `env` (BLBRS_* name -> value) and put every knob an
    earlier call set, and `env` does not name, back to its starting value."""
    for name in list(_KNOB_START):
        if name not in env:
            set_tuning(name, _KNOB_START[name])
    for name, value in env.items():
        if name not in _KNOB_START:
            _KNOB_START[name] = get_tuning(name)
        set_tuning(name, int(value))


def table_fault_take(device: int = 0):
    """The recorded pointer-table fault of `device`'s asynchronous *_dev_ptrs calls (read and
    cleared; synchronize the stream first), or None.  blbrs_table_fault_take."""
    out, found = _lib.TableFault(), ctypes.c_int(0)
    _check(_lib.load().blbrs_table_fault_take(int(device), ctypes.byref(out), ctypes.byref(found)))
    return {f: int(getattr(out, f)) for f, _ in out._fields_} if found.value else None


def debug_corrupt_next_table(slot: int) -> None:
    """Test hook: the next tagged pointer-table upload carries a wrong tag in entry `slot`."""
    _check(_lib.load().blbrs_debug_corrupt_next_table(int(slot)))


def rtc_stats() -> dict:
    st = _lib.RtcStats()
    _check(_lib.load().blbrs_rtc_get_stats(ctypes.byref(st)))
    return {f: (float(getattr(st, f)) if f == "compile_ms" else int(getattr(st, f))) for f, _ in st._fields_}


def rtc_wait(timeout_ms: int = -1) -> bool:
    """Wait for queued run-time networks to compile; False on timeout.  A compiled network is
    loaded by the next launch of its pass, in the launching thread."""
    rc = _lib.load().blbrs_rtc_wait(int(timeout_ms))
    if rc == ErrLimit.code:
        return False
    _check(rc)
    return True


def rtc_eligible(k: int, rows: int) -> bool:
    """Whether a decode pass of `rows` rows over k inputs takes a run-time network under the
    current knobs (rtc.hpp eligible(): BLBRS_RTC on, rows >= 2, k + rows > BLBRS_RTC_WIDE)."""
    return (get_tuning("BLBRS_RTC") != 0 and get_tuning("BLBRS_BITSLICE") != 0 and 2 <= k <= 16
            and 2 <= rows <= 8 and k + rows > get_tuning("BLBRS_RTC_WIDE"))


def rtc_network_source(coef: np.ndarray) -> tuple[str, int]:
    """(device source, VALU ops per 8-dword group) of the network for a rows x k coefficient
    matrix."""
    c = np.ascontiguousarray(coef, dtype=np.uint8)
    rows, k = c.shape
    buf = ctypes.create_string_buffer(1 << 20)
    ops = ctypes.c_int(0)
    _check(_lib.load().blbrs_rtc_network_source(k, rows, c.ctypes.data, buf, len(buf), ctypes.byref(ops)))
    return buf.value.decode(), int(ops.value)


def rtc_compile(coef: np.ndarray, mode: int = 0, strided: bool = True) -> bytes:
    """Compile (no device needed) the network kernel of a rows x k coefficient matrix and return
    its code object (AMDGPU ELF); raises ErrHIP with the compiler log on failure."""
    c = np.ascontiguousarray(coef, dtype=np.uint8)
    rows, k = c.shape
    n = ctypes.c_size_t(0)
    lib = _lib.load()
    _check(lib.blbrs_rtc_compile(k, rows, c.ctypes.data, int(mode), int(strided), None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value)
    _check(lib.blbrs_rtc_compile(k, rows, c.ctypes.data, int(mode), int(strided), buf, n.value, ctypes.byref(n)))
    return buf.raw[:n.value]


def version() -> str:
    return _lib.load().blbrs_version().decode()
