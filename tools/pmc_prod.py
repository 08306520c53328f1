"""PMC driver for the PRODUCTION library (blb_amd/libblbrs.so as bench.py loads it), run under
`rocprofv3 --pmc ...` (and once under --kernel-trace) by tools/pmc_prod.sh.

Every op below runs once untimed (warm-up: first-touch of the buffers, run-time network
compiled, code objects loaded) and then REPS times; tools/pmc_prod_summary.py averages the
counters and kernel-trace durations over the REPS launches, so each kernel's figures describe
a warm launch, as bench.py's HIP events do.  Calibration kernels of known traffic run first in
the same process:

  calib_copy        torch copy_ of 8 GiB (reads 8 GiB, writes 8 GiB)
  encode            EncodeBatch, RS(6,3) B=1024 x 8 MiB          (rs_code_kernel, store)
  reconstruct_data1 ReconstructBatch, data shard 1 missing        (rs_code_kernel, 1 row)
  verify            VerifyBatch                                   (rs_code_kernel, verify)
  encode_crc_65532  EncodeBatchCRC(65532)                         (encode_crc_tile_kernel + combine)
  crc32c_65532      ChecksumBatch of parity shard k, 65532 blocks (crc_stream_kernel)
  pack_tracts       PackPieces of B 8 MiB pieces from distinct tract sources (pack_kernel)
  pack_encode_rs6_3_distinct  PackEncode of all B*k data pieces, distinct sources (pack_encode_kernel)
  pack_encode_rs8_3_distinct  the same at RS(8,3) B=512
  then RS(12,5) B=480 (the bench's recovery batch): EncodeBatch and EncodeBatchCRC(65532) on the
  compiled network, a VerifyBatch, and blb's recovery shapes with the shipped default knobs (the
  pass's run-time network, compiled in the background after a first call on tables): the RPC
  with 1 and 5 bad data pieces (the first 12 good pieces read, all 5 absent slots rebuilt) and
  the client's 5-row ReconstructData; then the same 1-bad RPC on the v_perm tables
  (BLBRS_RTC = 0).

Prints the op plan (label, kernel-name needle, launches) and the libblbrs.so sha256 as one
JSON line; the summary consumes dispatches op by op in that order."""
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from blb_amd import _lib  # noqa: E402
from blb_amd import checksum, pack  # noqa: E402
from blb_amd import reedsolomon as rs  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
import tract_layout as TL  # noqa: E402

REPS = int(os.environ.get("PMC_REPS", "3"))
k, m, B, S = 6, 3, 1024, 8 << 20
dev = torch.device("cuda:0")
plan = []


def op(label, needle, fn, algo, **extra):
    """Warm-up + REPS launches of fn, each followed by a device sync (one dispatch at a time
    under the counters)."""
    for _ in range(1 + REPS):
        fn()
        torch.cuda.synchronize()
    plan.append({"label": label, "needle": needle, "launches": 1 + REPS, "algorithmic_bytes": algo, **extra})


def check(label, needle, fn):
    """One untimed launch the summary steps over (a verification between ops)."""
    r = fn()
    torch.cuda.synchronize()
    plan.append({"label": label, "needle": needle, "launches": 1, "skip": True, "algorithmic_bytes": 0})
    return r


src = torch.empty(8 << 30, dtype=torch.uint8, device=dev)
dst = torch.empty_like(src)
src.fill_(1)
torch.cuda.synchronize()
dst.copy_(src)  # calib_copy
torch.cuda.synchronize()
del src, dst
torch.cuda.empty_cache()

st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(97531)
st[:, :k].random_(0, 256, generator=g)
enc = rs.New(k, m)
torch.cuda.synchronize()
op("encode", "rs_code_kernel", lambda: enc.EncodeBatch(st), B * (k + m) * S)
op("reconstruct_data1", "rs_code_kernel",
   lambda: enc.ReconstructBatch(st, [i != 1 for i in range(k + m)], data_only=True), B * (k + 1) * S)
oks = []
op("verify", "rs_code_kernel", lambda: oks.append(enc.VerifyBatch(st)), B * (k + m) * S)
op("encode_crc_65532", "encode_crc_tile_kernel", lambda: enc.EncodeBatchCRC(st, 65532), B * (k + m) * S)
op("crc32c_65532", "crc_stream_kernel", lambda: checksum.ChecksumBatch(st[:, k], 65532), B * S)
# PackTracts into data shard 0 of every stripe (B pieces of 8 MiB): tracts of 64 KiB..8 MiB at
# padToLength offsets, every tract its own source bytes (end to end in a shuffled order, so
# no read is served by another tract's cached lines; tools/tract_layout.py).
prng = np.random.default_rng(17)
lay = TL.layout(B, S, prng)
pool, starts = TL.distinct_sources(lay, dev, g, prng, jitter=True)  # as rounds 3-4
pack_ext = TL.extents(lay, pool, starts)
pack_read = sum(ln for _, _, ln in lay)
torch.cuda.synchronize()
op("pack_tracts", "pack_kernel", lambda: pack.PackPieces(st[:, 0], S, pack_ext), pack_read + B * S,
   pieces=B, bytes_read=pack_read, bytes_written=B * S)
del pool, pack_ext
torch.cuda.empty_cache()
# PackTracts fused with Encode (curator encPack -> encEncode in one pass): every data
# piece of every stripe packed from distinct tract sources, parity encoded from registers.
lay = TL.layout(B * k, S, np.random.default_rng(29))
pool, starts = TL.distinct_sources(lay, dev, g, prng)
pe_ext = TL.extents(lay, pool, starts)
pe_read = sum(ln for _, _, ln in lay)
torch.cuda.synchronize()
op("pack_encode_rs6_3_distinct", "pack_encode_kernel", lambda: pack.PackEncode(enc, st, pe_ext),
   pe_read + B * (k + m) * S, pieces=B * k, tracts=len(lay), bytes_read=pe_read, bytes_written=B * (k + m) * S)
pe_ok = bool(check("verify_after_pack_encode_rs6_3", "rs_code_kernel", lambda: enc.VerifyBatch(st)).all())
del pool, pe_ext
torch.cuda.empty_cache()
verify_ok = bool(oks[-1].all()) and pe_ok
del st, oks
torch.cuda.empty_cache()

# blb's COLD class RS(8,3) (storage_class_loop.go:41-44), B=512: PackTracts fused with Encode from
# distinct tract sources.
k3, m3, B3 = 8, 3, 512
st = torch.empty((B3, k3 + m3, S), dtype=torch.uint8, device=dev)
enc3 = rs.New(k3, m3)
lay = TL.layout(B3 * k3, S, np.random.default_rng(83))
pool, starts = TL.distinct_sources(lay, dev, g, prng)
pe_ext = TL.extents(lay, pool, starts)
pe_read = sum(ln for _, _, ln in lay)
torch.cuda.synchronize()
op("pack_encode_rs8_3_distinct", "pack_encode_kernel", lambda: pack.PackEncode(enc3, st, pe_ext),
   pe_read + B3 * (k3 + m3) * S, pieces=B3 * k3, tracts=len(lay), bytes_read=pe_read,
   bytes_written=B3 * (k3 + m3) * S)
verify_ok = verify_ok and bool(check("verify_after_pack_encode_rs8_3", "rs_code_kernel", lambda: enc3.VerifyBatch(st)).all())
del pool, pe_ext, st
torch.cuda.empty_cache()

# blb's widest class: encode and encode fused with the ChecksumFile CRCs on the compiled
# bit-plane network, verify, and the recovery RPC shape on its run-time network.
k2, m2, B2 = 12, 5, 480
n2 = k2 + m2
st = torch.empty((B2, n2, S), dtype=torch.uint8, device=dev)
st[:, :k2].random_(0, 256, generator=g)
enc2 = rs.New(k2, m2)
torch.cuda.synchronize()
wb = B2 * n2 * S
op("encode_rs12_5_network", "rs_code_kernel", lambda: enc2.EncodeBatch(st), wb)
op("encode_crc_rs12_5_network", "encode_crc_tile_kernel", lambda: enc2.EncodeBatchCRC(st, 65532), wb)
oks2 = []
op("verify_rs12_5_network", "rs_code_kernel", lambda: oks2.append(enc2.VerifyBatch(st)), wb)
spread = [1 + (i * k2) // m2 for i in range(m2)]   # bench.py recovery_extras' bad pieces


def first_k_good(bad):
    good = [i for i in range(n2) if i not in bad]
    return [i in good[:k2] for i in range(n2)]


rpc1, rpc5 = first_k_good(spread[:1]), first_k_good(spread)
ok2 = bool(oks2[-1].all())
for label, present, data_only, rows in (("rpc_1bad_rs12_5", rpc1, False, m2), ("rpc_5bad_rs12_5", rpc5, False, m2),
                                        ("client_rows5_rs12_5", rpc5, True, m2)):
    # The shipped default (BLBRS_RTC = 1): the first call runs the tables and requests the pass's
    # network, compiled in the background; once compiled the op's launches run the network.
    check(f"request_network_{label}", "rs_code_kernel",
          lambda p=present, d=data_only: enc2.ReconstructBatch(st, p, data_only=d))
    rs.rtc_wait(120000)
    op(label, "rs_code_kernel", lambda p=present, d=data_only: enc2.ReconstructBatch(st, p, data_only=d),
       B2 * (k2 + rows) * S, present=[i for i in range(n2) if present[i]], knobs="shipped default (run-time network)")
    ok2 = ok2 and bool(check(f"verify_after_{label}", "rs_code_kernel", lambda: enc2.VerifyBatch(st)).all())
with rs.tuning(BLBRS_RTC=0):
    op("rpc_1bad_rs12_5_tables", "rs_code_kernel", lambda: enc2.ReconstructBatch(st, rpc1), wb,
       present=[i for i in range(n2) if rpc1[i]], knobs="BLBRS_RTC=0")
ok2 = ok2 and bool(enc2.VerifyBatch(st).all())
lib = _lib.LIB_PATH
print(json.dumps({"lib": lib, "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
                  "verify_ok": verify_ok, "k": k, "m": m, "batch": B, "shard": S, "reps": REPS, "plan": plan,
                  "wide": {"k": k2, "m": m2, "batch": B2, "compiled_network": enc2.compiled_network(),
                           "verify_ok": ok2}, "rtc": rs.rtc_stats()}))
