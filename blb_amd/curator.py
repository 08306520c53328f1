"""Curator drivers of the RS path (control only; no byte work): a restatement of how the
curator builds RSEncode requests.

  * encode_request -- tractPacker.encEncode (internal/curator/pack_tracts.go:277-292):
    N data pieces -> M parity pieces, IndexMap = nil, length = RSPieceLength.
  * reconstruct_request -- Curator.reconstructChunk (internal/curator/reconstruct.go:15-104):
    srcs = first n good pieces in index order, dests = replacements for bad indexes padded
    to m with (id 0, host "", index -1), IndexMap = srcIdx ++ dstIdx.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional, Sequence

from .blbcore import RS_PIECE_LENGTH, Error, RSChunkID, TSAddr


@dataclass
class RSEncodeReq:
    """core.RSEncodeReq (internal/core/tractserver_messages.go:147-154)."""
    tsid: int
    chunk_id: RSChunkID
    length: int
    srcs: list
    dests: list
    index_map: Optional[list]


def encode_request(chunk: RSChunkID, data_hosts: Sequence[TSAddr], parity_hosts: Sequence[TSAddr],
                   length: int = RS_PIECE_LENGTH) -> RSEncodeReq:
    """The replicated -> RS transition's RPC: sent to the first parity host."""
    return RSEncodeReq(parity_hosts[0].id, chunk, length, list(data_hosts), list(parity_hosts), None)


def reconstruct_request(chunk: RSChunkID, n: int, hosts: Sequence[TSAddr], bad_ids: Sequence[int],
                        allocate: Callable[[int], Optional[list]],
                        length: int = RS_PIECE_LENGTH) -> tuple[Optional[RSEncodeReq], Error]:
    """reconstruct.go:15-104.  `hosts` are the chunk's n+m pieces (data then parity);
    `allocate(count)` returns `count` replacement TSAddrs or None."""
    m = len(hosts) - n
    ok, ok_idx, dst_idx = [], [], []
    for i, h in enumerate(hosts):
        if h.id in bad_ids:
            dst_idx.append(i)
        else:
            ok.append(h)
            ok_idx.append(i)
    if len(ok) < n:
        return None, Error.ErrAllocHost
    if not dst_idx:
        return None, Error.ErrInvalidArgument
    srcs, src_idx = ok[:n], ok_idx[:n]
    new = allocate(len(dst_idx))
    if new is None:
        return None, Error.ErrAllocHost
    dests = list(new)
    while len(dests) < m:
        dests.append(TSAddr(0, ""))
        dst_idx.append(-1)
    return RSEncodeReq(dests[0].id, chunk, length, srcs, dests, src_idx + dst_idx), Error.NoError
