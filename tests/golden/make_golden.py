#!/usr/bin/env python3
"""Regenerate tests/golden/ from the REFERENCE struct_pack.

Runs oracle/_ref/golden_gen (compiled by `make -C oracle ref` from the
unmodified headers under /root/reference/include) and records:
  kat.json        type literals / type codes of every record type
  manifest.json   one entry per fixture: case, mode, n, seed, param, conf,
                  wire length, sha256 of the wire (and of the mode-B message
                  lengths); small fixtures also keep the wire as <name>.bin
  errs.json       mutation tests: base wire + edits → reference errc,
                  consume_len and canonical re-encoding of the decoded value
The inputs are NOT stored: they are regenerated from (case, n, seed, param)
by yalantinglibs_amd/synth.py (CPU) or spk_synth (GPU).

Usage: python tests/golden/make_golden.py [--big]
"""
import argparse
import hashlib
import json
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
GEN = os.path.join(ROOT, "oracle", "_ref", "golden_gen")

SEED = {"rec64": 0x5EED0002, "recs": 0x5EED0003, "outer": 0x5EED0004,
        "pad": 0x5EED0005, "mixed": 0x5EED0006, "rect": 0, "rpcrect": 0x5EED0007,
        "person": 0x5EED0008, "ints": 0x5EED0009, "opt": 0x5EED000A, "optp": 0x5EED000B,
        "var": 0x5EED000C, "varp": 0x5EED000D, "tags": 0x5EED000E, "group": 0x5EED000F,
        "deep": 0x5EED0010, "vnt": 0x5EED0011, "al8": 0x5EED0012, "alout": 0x5EED0013,
        "packed": 0x5EED0014, "alrec": 0x5EED0015,
        # one seed for the three writer versions of Cmp (same records)
        "cmp": 0x5EED0016, "cmpold": 0x5EED0016, "cmpnew": 0x5EED0016,
        "fv": 0x5EED0017, "fve": 0x5EED0018, "fv32": 0x5EED0019, "ev": 0x5EED001A,
        "valreq": 0x5EED001B, "exp": 0x5EED001C, "cmpg": 0x5EED001D, "monster": 0x5EED001E,
        "rect2": 0x5EED001F, "lists": 0x5EED0020, "maps": 0x5EED0021, "cplx": 0,
        "widet": 0x5EED0022, "wide": 0x5EED0023}

# (case_mode, n, param, conf, keep_bin)
SMALL = [
    ("rect_A", 1000, 0, "default"), ("rect_A", 20, 0, "default"),
    ("rect_A", 0, 0, "default"), ("rect_B", 10, 0, "default"),
    ("rec64_A", 0, 0, "default"), ("rec64_A", 1, 0, "default"),
    ("rec64_A", 255, 0, "default"), ("rec64_A", 256, 0, "default"),
    ("rec64_A", 1000, 0, "default"), ("rec64_A", 1000, 0, "typeinfo"),
    ("rec64_A", 1000, 0, "nometa"), ("rec64_A", 200, 0, "nometa"),
    ("rec64_B", 300, 0, "default"), ("rec64_B", 50, 0, "typeinfo"),
    ("rec64_B", 50, 0, "nometa"),
    ("recs_A", 0, 48, "default"), ("recs_A", 1, 48, "default"),
    ("recs_A", 100, 48, "default"), ("recs_A", 300, 48, "default"),
    ("recs_A", 3000, 48, "default"), ("recs_A", 40, 300, "default"),
    ("recs_A", 300, 48, "typeinfo"), ("recs_A", 300, 48, "nometa"),
    ("recs_A", 100, 48, "nometa"),
    ("recs_B", 500, 300, "default"), ("recs_B", 200, 48, "typeinfo"),
    ("recs_B", 100, 48, "nometa"),
    ("outer_A", 0, 16, "default"), ("outer_A", 1, 16, "default"),
    ("outer_A", 100, 16, "default"), ("outer_A", 1000, 16, "default"),
    ("outer_A", 30, 400, "default"), ("outer_B", 300, 16, "default"),
    ("outer_B", 40, 400, "default"),
    ("pad_A", 1000, 0, "default"), ("pad_B", 100, 0, "default"),
    ("mixed_A", 200, 40, "default"), ("mixed_A", 50, 400, "default"),
    ("mixed_B", 200, 300, "default"), ("mixed_A", 60, 40, "typeinfo"),
    ("rpcrect_A", 100, 0, "default"), ("rpcrect_B", 100, 0, "default"),
    ("person_A", 100, 64, "default"), ("person_B", 100, 300, "default"),
    ("ints_B", 100, 300, "default"), ("ints_B", 20, 3000, "default"),
    ("opt_A", 0, 16, "default"), ("opt_A", 1, 16, "default"),
    ("opt_A", 300, 16, "default"), ("opt_A", 40, 400, "default"),
    ("opt_A", 100, 48, "typeinfo"), ("opt_B", 200, 300, "default"),
    ("optp_A", 300, 0, "default"), ("optp_B", 200, 0, "default"),
    ("optp_B", 50, 0, "typeinfo"), ("optp_A", 20, 0, "nometa"),
    ("var_A", 0, 16, "default"), ("var_A", 1, 16, "default"),
    ("var_A", 300, 16, "default"), ("var_A", 40, 400, "default"),
    ("var_A", 100, 48, "typeinfo"), ("var_B", 200, 300, "default"),
    ("var_A", 3000, 8, "default"), ("var_A", 50, 8, "nometa"),
    ("varp_A", 300, 0, "default"), ("varp_B", 200, 0, "default"),
    ("varp_B", 50, 0, "typeinfo"), ("varp_A", 20, 0, "nometa"),
    # containers of non-trivially-serializable elements (SPK_OP_ARRAY)
    ("tags_A", 0, 4, "default"), ("tags_A", 1, 4, "default"),
    ("tags_A", 200, 6, "default"), ("tags_A", 30, 300, "default"),
    ("tags_B", 200, 6, "default"), ("tags_B", 20, 300, "default"),
    ("tags_A", 100, 6, "typeinfo"), ("tags_A", 50, 6, "nometa"),
    ("group_A", 0, 5, "default"), ("group_A", 100, 5, "default"),
    ("group_B", 100, 5, "default"), ("group_A", 3, 300, "default"),
    ("deep_A", 100, 4, "default"), ("deep_B", 100, 4, "default"),
    ("deep_A", 20, 300, "default"), ("deep_B", 30, 4, "nometa"),
    # std::variant members (SPK_OP_VARIANT), also inside a vector element
    ("vnt_A", 0, 6, "default"), ("vnt_A", 1, 6, "default"), ("vnt_A", 200, 6, "default"),
    ("vnt_B", 200, 6, "default"), ("vnt_A", 40, 300, "default"),
    ("vnt_A", 50, 6, "typeinfo"), ("vnt_B", 60, 6, "nometa"),
    # alignment overrides: alignas(8), nested alignas(4/8/16), #pragma pack(1) +
    # pack_alignment_v = 1, and a non-trivial record holding all three
    ("al8_A", 300, 0, "default"), ("al8_B", 50, 0, "default"), ("al8_A", 40, 0, "typeinfo"),
    ("alout_A", 300, 0, "default"), ("alout_B", 50, 0, "default"),
    ("alout_A", 40, 0, "typeinfo"), ("packed_A", 300, 0, "default"),
    ("packed_B", 50, 0, "default"), ("packed_A", 40, 0, "typeinfo"),
    ("alrec_A", 200, 20, "default"), ("alrec_B", 100, 20, "default"),
    ("alrec_A", 40, 20, "typeinfo"),
    # struct_pack::compatible members: total-length field of 2 and 4 bytes,
    # and the older / newer writers of the same type code
    ("cmp_A", 0, 8, "default"), ("cmp_A", 1, 8, "default"), ("cmp_A", 200, 8, "default"),
    ("cmp_A", 40, 300, "default"), ("cmp_A", 50, 8, "typeinfo"), ("cmp_B", 200, 8, "default"),
    ("cmp_B", 30, 300, "default"), ("cmp_A", 3000, 30, "default"),
    ("cmpold_A", 200, 8, "default"), ("cmpold_B", 100, 8, "default"),
    ("cmpnew_A", 200, 8, "default"), ("cmpnew_B", 100, 8, "default"),
    # sp_config USE_FAST_VARINT / ENCODING_WITH_VARINT records
    ("fv_A", 0, 8, "default"), ("fv_A", 1, 8, "default"), ("fv_A", 300, 8, "default"),
    ("fv_A", 40, 300, "default"), ("fv_A", 50, 8, "typeinfo"), ("fv_B", 300, 8, "default"),
    ("fv_A", 30, 8, "nometa"), ("fve_A", 300, 8, "default"), ("fve_B", 200, 8, "default"),
    ("fv32_A", 300, 0, "default"), ("fv32_B", 200, 0, "default"),
    ("ev_A", 300, 8, "default"), ("ev_B", 200, 8, "default"), ("ev_A", 30, 8, "nometa"),
    # optional / expected / compatible of values that are not trivially
    # serializable: the coro_rpc benchmark's ValidateRequest, expected<T, E>
    ("valreq_A", 0, 16, "default"), ("valreq_A", 1, 16, "default"),
    ("valreq_A", 300, 16, "default"), ("valreq_A", 40, 300, "default"),
    ("valreq_A", 50, 16, "typeinfo"), ("valreq_B", 200, 16, "default"),
    ("valreq_B", 40, 16, "nometa"), ("exp_A", 0, 16, "default"), ("exp_A", 300, 16, "default"),
    ("exp_B", 200, 16, "default"), ("exp_A", 50, 16, "typeinfo"), ("exp_A", 30, 300, "default"),
    ("cmpg_A", 0, 8, "default"), ("cmpg_A", 200, 8, "default"), ("cmpg_B", 200, 8, "default"),
    ("cmpg_A", 40, 300, "default"), ("cmpg_A", 50, 8, "typeinfo"),
    # the reference benchmark's Monster (20 of them: its OBJECT_COUNT) and
    # rect2<int32_t> with its ADL sp_config (fast varints, no meta info)
    ("monster_A", 0, 20, "default"), ("monster_A", 1, 20, "default"),
    ("monster_A", 20, 20, "default"), ("monster_A", 300, 20, "default"),
    ("monster_B", 200, 20, "default"), ("monster_A", 40, 300, "default"),
    ("monster_A", 50, 20, "typeinfo"), ("monster_B", 30, 20, "nometa"),
    ("rect2_A", 0, 0, "default"), ("rect2_A", 20, 0, "default"), ("rect2_A", 300, 0, "default"),
    ("rect2_B", 200, 0, "default"),
    # list / deque / map / set / multimap / multiset; the reference's
    # complicated_object (its cplx_B n1 typeinfo / default fixtures are the
    # reference's own binary goldens, tests/golden/ref_test_cross_platform*.dat)
    ("lists_A", 0, 6, "default"), ("lists_A", 1, 6, "default"), ("lists_A", 200, 6, "default"),
    ("lists_A", 30, 300, "default"), ("lists_B", 200, 6, "default"),
    ("lists_A", 50, 6, "typeinfo"), ("maps_A", 0, 0, "default"), ("maps_A", 1, 0, "default"),
    ("maps_A", 200, 0, "default"), ("maps_B", 200, 0, "default"), ("maps_A", 50, 0, "typeinfo"),
    ("cplx_B", 1, 0, "default"), ("cplx_B", 1, 0, "typeinfo"), ("cplx_A", 3, 0, "default"),
    ("cplx_A", 2, 0, "typeinfo"), ("cplx_B", 5, 0, "nometa"),
    # opt-in types (STRUCT_PACK_ENABLE_INT128 / _UNPORTABLE_TYPE): __int128,
    # std::bitset, wchar_t, u16string / u32string / wstring
    ("widet_A", 0, 0, "default"), ("widet_A", 300, 0, "default"), ("widet_B", 50, 0, "default"),
    ("widet_A", 40, 0, "typeinfo"), ("wide_A", 0, 6, "default"), ("wide_A", 1, 6, "default"),
    ("wide_A", 200, 6, "default"), ("wide_B", 100, 6, "default"), ("wide_A", 40, 300, "default"),
    ("wide_A", 50, 6, "typeinfo"), ("wide_B", 30, 6, "nometa"),
]
MEDIUM = [  # digest only (wire > ~1 MB)
    ("rec64_A", 65535, 0, "default"), ("rec64_A", 65536, 0, "default"),
    ("rec64_A", 70000, 0, "default"), ("recs_A", 70000, 48, "default"),
    ("outer_A", 70000, 16, "default"), ("mixed_A", 20000, 40, "default"),
    ("recs_B", 70000, 48, "default"), ("outer_B", 70000, 16, "default"),
    ("ints_B", 3, 70000, "default"), ("ints_B", 20, 70000, "default"),
    ("opt_A", 70000, 48, "default"), ("optp_A", 70000, 0, "default"),
    ("opt_B", 70000, 48, "default"),
    ("var_A", 70000, 48, "default"), ("varp_A", 70000, 0, "default"),
    ("var_B", 70000, 48, "default"),
    ("tags_A", 70000, 6, "default"), ("tags_B", 20000, 6, "default"),
    ("group_A", 20000, 5, "default"), ("deep_A", 20000, 4, "default"),
    ("vnt_A", 30000, 8, "default"), ("vnt_B", 20000, 8, "default"),
    ("cmp_A", 30000, 48, "default"), ("cmp_B", 20000, 48, "default"),
    ("fv_A", 70000, 48, "default"), ("fve_B", 20000, 16, "default"),
    ("ev_A", 70000, 16, "default"),
    ("recs_A", 200, 20000, "default"), ("outer_A", 100, 2000, "default"),
    ("valreq_A", 30000, 16, "default"), ("valreq_B", 20000, 16, "default"),
    ("exp_A", 30000, 16, "default"), ("cmpg_A", 30000, 16, "default"),
    ("cmpg_B", 20000, 16, "default"), ("monster_A", 30000, 20, "default"),
    ("monster_B", 20000, 20, "default"), ("rect2_A", 70000, 0, "default"),
    ("lists_A", 30000, 6, "default"), ("maps_A", 20000, 0, "default"),
    ("maps_B", 10000, 0, "default"), ("cplx_A", 3000, 0, "default"),
    ("wide_A", 20000, 16, "default"), ("widet_A", 30000, 0, "default"),
]
BIG = [  # BASELINE.json full-size configs (digest only)
    ("rec64_A", 100_000_000, 0, "default"),
    ("recs_A", 10_000_000, 48, "default"),
    ("outer_A", 10_000_000, 16, "default"),
    ("rec64_B", 1_000_000, 0, "default"),
    ("recs_B", 1_000_000, 48, "default"),
]


# coro_rpc framed batches: (case_B, n, param, req|resp, function name, seq_base)
FRAMES = [
    ("rpcrect_B", 100, 0, "req", "echo_rect", 1), ("rpcrect_B", 100, 0, "resp", "", 1),
    ("person_B", 120, 48, "req", "echo_person", 7), ("person_B", 120, 48, "resp", "", 7),
    ("ints_B", 20, 1000, "req", "array_1K_int", 0xFFFFFFF0),
    ("ints_B", 20, 1000, "resp", "", 0xFFFFFFF0), ("rec64_B", 40, 0, "req", "echo_rec64", 0),
]


# full-size C5 frames (bench.py --config c5: 333,333 messages per type): digests only
FRAMES_BIG = [
    ("rpcrect_B", 333333, 0, "req", "echo_rect", 0), ("rpcrect_B", 333333, 0, "resp", "", 0),
    ("person_B", 333333, 48, "req", "echo_person", 0), ("person_B", 333333, 48, "resp", "", 0),
    ("ints_B", 333333, 2000, "req", "array_1K_int", 0), ("ints_B", 333333, 2000, "resp", "", 0),
]


def func_id(name):
    """router.hpp:121-127: MD5Hash32Constexpr(function name)"""
    return int.from_bytes(hashlib.md5(name.encode()).digest()[:4], "big") if name else 0


def make_frames(tmp, big=False):
    out = []
    for cm, n, param, kind, fname, seq in FRAMES + (FRAMES_BIG if big else []):
        case = cm[:-2]
        name = f"frames_{case}_{kind}_n{n}_p{param}"
        keep = (cm, n, param, kind, fname, seq) in FRAMES
        d = HERE if keep else tmp
        wire = os.path.join(d, name + ".bin")
        lens = os.path.join(d, name + ".lens")
        fid = func_id(fname)
        subprocess.run([GEN, "frames", cm, str(n), str(SEED[case]), str(param), kind, str(fid),
                        str(seq), wire, lens], check=True, stdout=subprocess.DEVNULL)
        ent = {"name": name, "case": case, "n": n, "seed": SEED[case], "param": param,
               "kind": kind, "function": fname, "function_id": fid, "seq_base": seq,
               "wire_len": os.path.getsize(wire), "sha256": sha256_file(wire),
               "lens_sha256": sha256_file(lens)}
        if keep:
            ent.update({"file": name + ".bin", "lens": name + ".lens"})
        else:
            os.remove(wire)
            os.remove(lens)
        out.append(ent)
    return out


def name_of(cm, n, param, conf):
    return f"{cm}_n{n}_p{param}_{conf}"


def sha256_file(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        while True:
            b = f.read(1 << 24)
            if not b:
                break
            h.update(b)
    return h.hexdigest()


def emit(cm, n, param, conf, keep_bin, tmp):
    case = cm[:-2]
    seed = SEED[case]
    wire = os.path.join(tmp, "wire.bin")
    lens = os.path.join(tmp, "lens.bin")
    subprocess.run([GEN, "emit", cm, str(n), str(seed), str(param), conf, wire, lens],
                   check=True, stdout=subprocess.DEVNULL)
    ent = {"name": name_of(cm, n, param, conf), "case": case, "mode": cm[-1],
           "n": n, "seed": seed, "param": param, "conf": conf,
           "wire_len": os.path.getsize(wire), "sha256": sha256_file(wire)}
    if cm.endswith("_B"):
        ent["lens_sha256"] = sha256_file(lens)
    if keep_bin:
        with open(wire, "rb") as f:
            data = f.read()
        with open(os.path.join(HERE, ent["name"] + ".bin"), "wb") as f:
            f.write(data)
        if cm.endswith("_B"):
            with open(lens, "rb") as f:
                ld = f.read()
            with open(os.path.join(HERE, ent["name"] + ".lens"), "wb") as f:
                f.write(ld)
        ent["file"] = ent["name"] + ".bin"
    os.remove(wire)
    if os.path.exists(lens):
        os.remove(lens)
    return ent


# ---- mutation tests -------------------------------------------------------
ERR_BASES = [
    ("recs_A", 5, 10, "default"), ("recs_A", 300, 48, "default"),
    ("rec64_A", 3, 0, "default"), ("recs_A", 3, 20, "typeinfo"),
    ("rect_A", 3, 0, "default"), ("outer_A", 4, 8, "default"),
    ("rec64_A", 300, 0, "default"), ("recs_B", 1, 300, "default"),
    ("rec64_B", 1, 0, "default"), ("mixed_A", 3, 300, "default"),
    ("opt_A", 6, 10, "default"), ("optp_B", 1, 0, "default"), ("opt_B", 1, 20, "default"),
    ("var_A", 6, 10, "default"), ("varp_B", 1, 0, "default"), ("varp_A", 4, 0, "default"),
    ("tags_A", 5, 4, "default"), ("tags_B", 1, 6, "default"), ("group_A", 4, 3, "default"),
    ("group_B", 1, 4, "default"), ("deep_A", 4, 3, "default"), ("deep_B", 1, 4, "default"),
    ("vnt_A", 6, 4, "default"), ("vnt_B", 1, 4, "default"), ("vnt_B", 1, 40, "default"),
    ("alout_A", 5, 0, "default"), ("packed_B", 1, 0, "default"), ("alrec_A", 4, 10, "default"),
    # width-8 container lengths (metainfo 0x18): no reference encoder writes
    # them below 2^32 elements, but every decoder must read them
    # (unpacker.hpp:572-619); the base is our width-8 re-encoding, decoded by
    # the reference
    ("recs_A", 5, 10, "default", 8), ("outer_A", 4, 8, "default", 8),
    ("recs_B", 1, 30, "default", 8), ("tags_A", 4, 4, "default", 8),
    ("mixed_A", 3, 20, "default", 4), ("recs_A", 4, 10, "default", 2),
    ("cmp_A", 6, 10, "default"), ("cmp_B", 1, 20, "default"), ("cmp_A", 3, 10, "typeinfo"),
    ("cmp_B", 1, 300, "default"),
    ("fv_A", 6, 10, "default"), ("fv_B", 1, 10, "default"), ("fve_A", 5, 6, "default"),
    ("fv32_A", 8, 0, "default"), ("fv32_B", 1, 0, "default"), ("ev_A", 5, 6, "default"),
    ("ev_B", 1, 6, "default"),
    ("valreq_A", 5, 10, "default"), ("valreq_B", 1, 10, "default"), ("valreq_A", 3, 10, "typeinfo"),
    ("exp_A", 6, 10, "default"), ("exp_B", 1, 10, "default"),
    ("cmpg_A", 6, 10, "default"), ("cmpg_B", 1, 10, "default"),
    ("monster_A", 4, 10, "default"), ("monster_B", 1, 10, "default"),
    ("rect2_A", 6, 0, "default"), ("rect2_B", 1, 0, "default"),
    ("lists_A", 5, 4, "default"), ("lists_B", 1, 6, "default"),
    ("maps_A", 4, 0, "default"), ("maps_B", 1, 0, "default"),
    ("wide_A", 4, 6, "default"), ("wide_B", 1, 6, "default"), ("widet_A", 3, 0, "default"),
]
# compatible members across writer versions: (writer, reader, n, param) — the
# writer's message mutated and decoded as the reader's type (one type code)
XERR_BASES = [
    ("cmpold_A", "cmp_A", 6, 10), ("cmpnew_A", "cmp_A", 6, 10), ("cmp_A", "cmpold_A", 6, 10),
    ("cmp_A", "cmpnew_A", 6, 10), ("cmpold_B", "cmp_B", 1, 10), ("cmpnew_B", "cmp_B", 1, 10),
    ("cmp_B", "cmpold_B", 1, 10),
]


def wide_wire(cm, n, param, conf, width):
    """The message golden_gen would emit, with every container length (and the
    outer vector count) written at `width` bytes and the metainfo byte saying
    so: header from spk_vector_header, body from the oracle's encode_body."""
    import ctypes as ct
    import numpy as np
    sys.path.insert(0, ROOT)
    from yalantinglibs_amd import _capi as C
    from yalantinglibs_amd import layout as LY
    from yalantinglibs_amd import schema as S
    from yalantinglibs_amd import synth
    case = cm[:-2]
    confv = {"default": S.DEFAULT, "typeinfo": S.ENABLE_TYPE_INFO,
             "nometa": S.DISABLE_ALL_META_INFO}[conf]
    L = LY.case_layout(case, confv)
    _, recs, heaps = synth.make_batch(case, n, SEED[case], param)
    o = C.load_oracle()
    hp = (ct.c_void_p * max(len(heaps), 1))(*[h.ctypes.data if h.size else 0 for h in heaps])
    rp = ct.c_void_p(recs.ctypes.data if n else 0)
    body = np.zeros(1 << 20, np.uint8)
    wr = ct.c_uint64()
    assert o.spko_encode_body(L.ptr, n, rp, hp, width, ct.c_void_p(body.ctypes.data),
                              body.size, ct.byref(wr)) == 0
    if cm.endswith("_B"):  # one message: the T header at this width
        assert n == 1
        lib = C.load_codec()
        vb = (ct.c_uint8 * 512)()
        k = lib.spk_vector_header(L.ptr, 0, width, vb, 512)
        hdr = bytes(vb[:k - width])  # fmt_vector's header: swap in fmt_one's code
        code = L.c.fmt_one.code
        hdr = bytes([(code & 0xFE) | (hdr[0] & 1)]) + code.to_bytes(4, "little")[1:] + hdr[4:]
        return hdr + body[:wr.value].tobytes()
    lib = C.load_codec()
    vb = (ct.c_uint8 * 512)()
    k = lib.spk_vector_header(L.ptr, n, width, vb, 512)
    assert k > 0
    return bytes(vb[:k]) + body[:wr.value].tobytes()


def mutations(wire_len, rng):
    muts = [f"trunc {i}" for i in range(0, min(wire_len, 48))]
    muts += [f"trunc {wire_len - d}" for d in (1, 2, 3, 7, 8, 9) if wire_len - d >= 48]
    for pos in range(min(wire_len, 12)):
        for v in (0x00, 0xFF, 0x01, 0x08, 0x10, 0x18, 0x04, 0x0C, 0x03):
            muts.append(f"set {pos} {v}")
    for _ in range(64):
        pos = rng.randrange(wire_len) if wire_len else 0
        muts.append(f"set {pos} {rng.randrange(256)}")
    for _ in range(16):
        pos = rng.randrange(wire_len) if wire_len else 0
        muts.append(f"set {pos} {rng.randrange(256)} trunc {rng.randrange(wire_len + 1)}")
    return muts


def make_errs(tmp):
    out = []
    for eb in ERR_BASES + [(r, n, p, "default", 0, w) for w, r, n, p in XERR_BASES]:
        cm, n, param, conf = eb[:4]
        width = eb[4] if len(eb) > 4 else 0
        writer = eb[5] if len(eb) > 5 else cm
        # each base's mutations from an RNG of its own key: adding a base never
        # changes the mutation sets of the others
        rng = random.Random(f"{cm}|{n}|{param}|{conf}|{width}|{writer}")
        case = cm[:-2]
        seed = SEED[case]
        wire = os.path.join(tmp, "ewire.bin")
        if width:
            with open(wire, "wb") as f:
                f.write(wide_wire(cm, n, param, conf, width))
        else:
            subprocess.run([GEN, "emit", writer, str(n), str(seed), str(param), conf, wire,
                            os.path.join(tmp, "elens.bin")], check=True,
                           stdout=subprocess.DEVNULL)
        with open(wire, "rb") as f:
            base = f.read()
        muts = mutations(len(base), rng)
        if width or writer != cm:  # the unmutated message first
            muts.insert(0, f"trunc {len(base)}")
        if case in ("var", "varp"):  # overlong / 10-byte / unterminated varints
            for p0 in range(0, min(len(base), 48), 3):
                run = " ".join(f"set {p0 + j} 255" for j in range(10))
                muts.append(run)
                muts.append(" ".join(f"set {p0 + j} 255" for j in range(9)) + f" set {p0 + 9} 1")
                muts.append(run + f" trunc {p0 + 6}")
        mfile = os.path.join(tmp, "muts.txt")
        with open(mfile, "w") as f:
            f.write("\n".join(muts) + "\n")
        res = subprocess.run([GEN, "errs", cm, str(n), str(seed), str(param), conf,
                              mfile, wire], check=True, capture_output=True, text=True)
        rows = [json.loads(line) for line in res.stdout.splitlines() if line.strip()]
        for r in rows:  # keep a digest of the canonical re-encoding, not the bytes
            re_hex = r.pop("reenc")
            r["reenc_sha256"] = (hashlib.sha256(bytes.fromhex(re_hex)).hexdigest()
                                 if re_hex is not None else None)
        assert len(rows) == len(muts), (cm, len(rows), len(muts))
        if width:
            assert rows[0]["errc"] == 0, (cm, width, rows[0])  # the reference reads it
        if writer != cm:
            assert rows[0]["errc"] == 0, (writer, cm, rows[0])
        out.append({"case": case, "mode": cm[-1], "n": n, "seed": seed, "param": param,
                    "conf": conf, "width": width or None, "writer": writer[:-2],
                    "base": base.hex(),
                    "tests": [{"mut": m, **r} for m, r in zip(muts, rows)]})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true", help="also the full-size configs")
    ap.add_argument("--errs-only", action="store_true", help="rewrite errs.json only")
    args = ap.parse_args()
    if args.errs_only:
        with tempfile.TemporaryDirectory() as tmp:
            errs = make_errs(tmp)
        with open(os.path.join(HERE, "errs.json"), "w") as f:
            json.dump(errs, f, indent=0)
        print(f"{sum(len(e['tests']) for e in errs)} mutation tests")
        return
    if not os.path.exists(GEN):
        sys.exit(f"{GEN} missing: run `make -C oracle ref` (needs /root/reference)")
    kat = json.loads(subprocess.run([GEN, "kat"], check=True, capture_output=True,
                                    text=True).stdout)
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1, sort_keys=True)
    man_path = os.path.join(HERE, "manifest.json")
    old = {}
    if os.path.exists(man_path):
        with open(man_path) as f:
            old = {e["name"]: e for e in json.load(f)}
    ents = []
    with tempfile.TemporaryDirectory() as tmp:
        for cm, n, p, c in SMALL:
            ents.append(emit(cm, n, p, c, True, tmp))
        for cm, n, p, c in MEDIUM:
            ents.append(emit(cm, n, p, c, False, tmp))
        for cm, n, p, c in BIG:
            nm = name_of(cm, n, p, c)
            if args.big:
                print("big:", nm, flush=True)
                ents.append(emit(cm, n, p, c, False, tmp))
            elif nm in old:
                ents.append(old[nm])
        for e in ents:
            e.setdefault("size_class", "big" if any(
                name_of(*b) == e["name"] for b in BIG) else "small")
        with open(man_path, "w") as f:
            json.dump(ents, f, indent=1)
        errs = make_errs(tmp)
        frames = make_frames(tmp, args.big)
        if not args.big:  # keep the full-size digests of an earlier --big run
            fp = os.path.join(HERE, "frames.json")
            if os.path.exists(fp):
                with open(fp) as f:
                    frames += [e for e in json.load(f) if "file" not in e]
    with open(os.path.join(HERE, "frames.json"), "w") as f:
        json.dump(frames, f, indent=1)
    with open(os.path.join(HERE, "errs.json"), "w") as f:
        json.dump(errs, f, indent=0)
    print(f"{len(ents)} fixtures, {sum(len(e['tests']) for e in errs)} mutation tests")


if __name__ == "__main__":
    main()
