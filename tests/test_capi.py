"""CPU-side tests of the C ABI (no compute calls need a GPU here):
  * libblbrs.so loads and exports every function include/blb_rs.h declares;
  * reedsolomon.New's argument errors and the encoding matrix match the oracle;
  * without a GPU the engine fails loudly (ErrNoDevice) -- there is no CPU fallback.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "blb_rs.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(blbrs_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from blb_amd import _lib
    lib = _lib.load()
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), f"libblbrs.so does not export {name}"
        assert name in _lib.SIGNATURES, f"ctypes signature missing for {name}"
    assert set(_lib.SIGNATURES) == set(declared)


_C_SIZES = {"uint64_t": 8, "int64_t": 8, "size_t": 8, "double": 8, "uint32_t": 4, "int32_t": 4, "int": 4}


def header_structs():
    """{typedef name: [(field, C type), ...]} of every plain typedef struct in the header."""
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for body, name in re.findall(r"typedef struct\s*\{(.*?)\}\s*(\w+)\s*;", text, flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            m = re.match(r"((?:const\s+)?\w+\s*\**)\s*(.*)", decl)
            ctype, names = m.group(1).strip(), m.group(2)
            for nm in names.split(","):
                nm = nm.strip()
                ptr = nm.startswith("*") or ctype.endswith("*")
                fields.append((nm.lstrip("*").strip(), "ptr" if ptr else ctype))
        out[name] = fields
    return out


def test_ctypes_structs_match_header():
    """Every ctypes mirror of a header struct (blb_amd/_lib.py) has the header's fields, in its
    order, and its size: a field added to the C side and not to the mirror would make every
    counter after it read the wrong bytes."""
    from blb_amd import _lib
    structs = header_structs()
    mirrors = [c for c in vars(_lib).values()
               if isinstance(c, type) and issubclass(c, ctypes.Structure) and (c.__doc__ or "").startswith("blbrs_")]
    assert len(mirrors) >= 6
    for cls in mirrors:
        fields = structs[cls.__doc__.strip()]
        assert [f for f, _ in cls._fields_] == [f for f, _ in fields], cls.__doc__
        size = 0
        for _, t in fields:
            w = 8 if t == "ptr" else _C_SIZES[t]
            size = (size + w - 1) // w * w + w
        size = (size + 7) // 8 * 8 if any(t == "ptr" or _C_SIZES.get(t) == 8 for _, t in fields) else size
        assert ctypes.sizeof(cls) == size, (cls.__doc__, ctypes.sizeof(cls), size)


def test_error_codes_match_header():
    from blb_amd import reedsolomon as rs
    text = open(HEADER).read()
    codes = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define (BLBRS_\w+)\s+\(?(-?\d+)\)?", text)}
    assert codes["BLBRS_ERR_INV_SHARD_NUM"] == rs.ErrInvShardNum.code
    assert codes["BLBRS_ERR_MAX_SHARD_NUM"] == rs.ErrMaxShardNum.code
    assert codes["BLBRS_ERR_TOO_FEW_SHARDS"] == rs.ErrTooFewShards.code
    assert codes["BLBRS_ERR_SHARD_NO_DATA"] == rs.ErrShardNoData.code
    assert codes["BLBRS_ERR_SHARD_SIZE"] == rs.ErrShardSize.code
    assert codes["BLBRS_ERR_NO_DEVICE"] == rs.ErrNoDevice.code


def test_new_errors_like_klauspost():
    from blb_amd import reedsolomon as rs
    with pytest.raises(rs.ErrInvShardNum):
        rs.New(0, 3)
    with pytest.raises(rs.ErrInvShardNum):
        rs.New(6, 0)
    with pytest.raises(rs.ErrInvShardNum):
        rs.New(-1, 2)
    with pytest.raises(rs.ErrMaxShardNum):
        rs.New(250, 7)
    enc = rs.New(250, 6)
    assert enc.Shards == 256


@pytest.mark.parametrize("k,m", [(3, 2), (4, 2), (6, 3), (8, 3), (10, 3), (10, 4), (12, 5), (20, 9)])
def test_engine_matrix_matches_oracle(oracle_lib, k, m):
    from blb_amd import reedsolomon as rs
    assert np.array_equal(rs.New(k, m).matrix(), oracle_lib.build_matrix(k, m))


def test_shard_checks_precede_device_use():
    """klauspost's argument errors come before any GPU work (they hold with no GPU)."""
    from blb_amd import reedsolomon as rs
    enc = rs.New(3, 2)
    S = 64
    with pytest.raises(rs.ErrTooFewShards):
        enc.Encode([np.zeros(S, np.uint8)] * 4)
    with pytest.raises(rs.ErrShardNoData):
        enc.Encode([np.zeros(0, np.uint8)] * 5)
    with pytest.raises(rs.ErrShardSize):
        enc.Encode([np.zeros(S, np.uint8)] * 4 + [np.zeros(S - 1, np.uint8)])
    with pytest.raises(rs.ErrTooFewShards):
        enc.Reconstruct([np.zeros(S, np.uint8), None, None, None, np.zeros(S, np.uint8)])
    # all present: no work, no device needed (klauspost returns nil)
    full = [np.zeros(S, np.uint8) for _ in range(5)]
    enc.Reconstruct(full)


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from blb_amd import reedsolomon as rs
    enc = rs.New(6, 3)
    sh = [np.ones(128, np.uint8) for _ in range(9)]
    with pytest.raises((rs.ErrNoDevice, rs.ErrHIP)):
        enc.Encode(sh)


def test_c_abi_null_arguments():
    from blb_amd import _lib
    lib = _lib.load()
    assert lib.blbrs_new(3, 2, None) == -7
    h = ctypes.c_void_p()
    assert lib.blbrs_new(3, 2, ctypes.byref(h)) == 0
    assert lib.blbrs_data_shards(h) == 3 and lib.blbrs_parity_shards(h) == 2
    assert lib.blbrs_encode(h, None, None) == -7
    small = (ctypes.c_uint8 * 4)()
    assert lib.blbrs_matrix(h, small, 4) == -7
    lib.blbrs_free(h)
    assert lib.blbrs_strerror(-3).decode() == "too few shards given"
    assert b"gfx950" in lib.blbrs_version()


def test_compiled_network_covers_blb_classes(knob):
    """The parity rows built into the library (gf_bitslice.hpp, constexpr buildMatrix) equal
    the runtime matrix for every compiled (k, m) -- with BLBRS_BITSLICE=2 Encode / Verify of
    all 30 shapes run the bit-plane network.  By default only the wide shapes do, each kernel
    with its own threshold (rs_code_kernel and PackTracts + Encode k + m > 9, the fused
    encode+CRC tile kernel k + m > 11); other shapes and BLBRS_BITSLICE=0 keep the v_perm
    table path.  Wide k outside the compiled list takes a run-time network (rtc) when opted in."""
    from blb_amd import reedsolomon as rs
    knob("BLBRS_BITSLICE", 2)
    for k in (3, 4, 6, 8, 10, 12):
        for m in range(1, 6):
            assert rs.New(k, m).compiled_network()["code"], (k, m)
    for k, m in ((5, 3), (10, 6), (2, 2), (20, 4)):
        assert not rs.New(k, m).compiled_network()["code"], (k, m)
    knob("BLBRS_BITSLICE", 1)
    nets = {(k, m): rs.New(k, m).compiled_network() for k, m in ((12, 5), (10, 4), (8, 3), (6, 3), (3, 2), (14, 4))}
    assert [nets[s]["code"] for s in ((12, 5), (10, 4), (8, 3), (6, 3), (3, 2))] == [True, True, True, False, False]
    assert [nets[s]["tile"] for s in ((12, 5), (10, 4), (8, 3), (6, 3))] == [True, True, False, False]
    assert [nets[s]["pack"] for s in ((12, 5), (10, 4), (8, 3), (6, 3))] == [True, True, True, False]
    # run-time networks compile in the background by default (BLBRS_RTC = 1): wide k outside the
    # compiled list takes one; BLBRS_RTC = 0 keeps it on tables
    assert nets[(14, 4)] == {"code": False, "tile": False, "pack": False, "rtc": True}
    knob("BLBRS_RTC", 0)
    assert rs.New(14, 4).compiled_network() == {"code": False, "tile": False, "pack": False, "rtc": False}
    knob("BLBRS_RTC", 1)
    assert not rs.New(12, 5).compiled_network()["rtc"]   # the compiled encode network wins
    knob("BLBRS_BITSLICE", 0)
    assert not any(rs.New(12, 5).compiled_network().values())


def test_one_hip_runtime_whatever_the_import_order():
    """torch's wheel carries its own libamdhip64 / libhsa-runtime64 under the SONAMEs libblbrs.so
    links.  Loading the library before torch used to map /opt/rocm's copies first and torch's
    second: two HIP runtimes over one /dev/kfd (the second found no device).  _lib.load() now
    brings torch's runtime in first, so one copy is mapped in either order."""
    import subprocess
    import sys
    from conftest import ROOT
    code = ("import sys; sys.path.insert(0, %r)\nfrom blb_amd import _lib\n_lib.load()\nimport torch\n"
            "maps = open('/proc/self/maps').read()\n"
            "print(sorted({l.split()[-1] for l in maps.splitlines() if 'libamdhip64' in l or 'libhsa-runtime64' in l}))"
            % ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, check=True).stdout
    libs = eval(out.strip().splitlines()[-1])  # a list literal printed above
    assert sum("libamdhip64" in x for x in libs) == 1 and sum("libhsa-runtime64" in x for x in libs) == 1, libs


@pytest.mark.gpu
def test_gpu_fault_watch_registers():
    """blbrs_debug_watch_faults registers its HSA system-event handler in the HSA runtime that HIP
    loaded: status 0, and again 0 (registered once per process)."""
    from blb_amd import _lib
    lib = _lib.load()
    assert lib.blbrs_debug_watch_faults() == 0, lib.blbrs_last_error()
    assert lib.blbrs_debug_watch_faults() == 0
