"""CPU: the C++20 front end (include/ylt/struct_pack_gpu.hpp and friends).

Compiles tests/cpp/test_type_code.cpp host-only (it static_asserts the
reference's type-code KATs at compile time) and checks its JSON against the
reference's KATs (tests/golden/kat.json) and the Python mirror's
descriptors (yalantinglibs_amd/layout.py): both front ends must hand the
C ABI identical descriptors."""
import json
import os
import subprocess

import pytest

import spk_helpers as H
from yalantinglibs_amd import layout as LY
from yalantinglibs_amd import schema as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang++"


@pytest.fixture(scope="module")
def cpp_json(tmp_path_factory):
    if not os.path.exists(CLANG):
        pytest.skip("clang++ not available")
    exe = str(tmp_path_factory.mktemp("cpp") / "ttc")
    subprocess.run([CLANG, "-std=c++20", "-O1", "-DNDEBUG", "-DSTRUCT_PACK_ENABLE_INT128",
                    "-DSTRUCT_PACK_ENABLE_UNPORTABLE_TYPE", "-I", os.path.join(ROOT, "include"),
                    "-o", exe, os.path.join(ROOT, "tests", "cpp", "test_type_code.cpp")],
                   check=True)
    return json.loads(subprocess.run([exe], check=True, capture_output=True, text=True).stdout)


def test_cpp_type_codes_match_reference_kats(cpp_json):
    kat = H.kat()
    for name, v in cpp_json["kat"].items():
        assert v["code"] == kat[name]["code"], name
        assert v["literal"] == kat[name]["literal"], name


@pytest.mark.parametrize("case,conf", [("rec64", 0), ("recs", 0), ("outer", 0), ("pad", 0),
                                       ("mixed", 0), ("rect", 0), ("rpcrect", 0),
                                       ("person", 0), ("ints", 0), ("opt", 0), ("optp", 0),
                                       ("var", 0), ("varp", 0), ("tags", 0), ("group", 0),
                                       ("deep", 0), ("vnt", 0), ("cmpg", 0), ("fv", 0),
                                       ("fve", 0), ("fv32", 0), ("ev", 0), ("valreq", 0),
                                       ("monster", 0), ("rect2", 0), ("lists", 0), ("maps", 0),
                                       ("alrec", 0), ("cmp", 0), ("cmpnew", 0),
                                       ("widet", 0), ("wide", 0),
                                       ("recs", S.ENABLE_TYPE_INFO),
                                       ("rec64", S.DISABLE_ALL_META_INFO)])
def test_cpp_and_python_descriptors_agree(cpp_json, case, conf):
    key = case + {0: "", S.ENABLE_TYPE_INFO: "_typeinfo", S.DISABLE_ALL_META_INFO: "_nometa"}[conf]
    c = cpp_json["layout"][key]
    L = LY.case_layout(case, conf).c
    assert c["flags"] == L.flags and c["stride"] == L.rec_stride
    assert c["ops"] == [[L.ops[i].kind, L.ops[i].rec_off, L.ops[i].size, L.ops[i].aux]
                        for i in range(L.n_ops)]
    assert c["vec"] == [L.fmt_vector.code, L.fmt_vector.flags, L.fmt_vector.literal_len]
    assert c["one"] == [L.fmt_one.code, L.fmt_one.flags, L.fmt_one.literal_len]


# ---- the front end compiles with the reference's toolchain and next to the
# reference headers (the coro_rpc drop-in case) --------------------------------
REF_INC = "/root/reference/include"


def _compile(cxx, src, extra=(), syntax_only=True):
    cmd = [cxx, "-std=c++20", "-DNDEBUG", "-I", os.path.join(ROOT, "include"), *extra]
    cmd += ["-fsyntax-only", "-x", "c++", "-"] if syntax_only else []
    return subprocess.run(cmd, input=src, capture_output=True, text=True)


USE_FRONT_END = """
#include <ylt/struct_pack_gpu.hpp>
struct person { int64_t id; std::string name; int age; double salary; };
struct refl_point { int x, y, z; };
YLT_REFL(refl_point, x, y, z);
struct with_varint { struct_pack::var_int32_t a; std::vector<int> b; };
void use() {
  std::vector<person> v;
  auto buf = struct_pack::gpu::serialize(v);
  auto r = struct_pack::gpu::deserialize<std::vector<person>>(buf);
  auto r2 = struct_pack::gpu::deserialize<struct_pack::sp_config::DEFAULT, person>(buf);
  std::size_t consumed = 0;
  person p;
  struct_pack::err_code ec = struct_pack::gpu::deserialize_to(p, buf, consumed);
  (void)r; (void)r2; (void)ec;
  static_assert(struct_pack::gpu::is_gpu_batch_v<std::vector<with_varint>>);
  static_assert(!struct_pack::gpu::detail::is_trivially_serializable<refl_point>());
  static_assert(struct_pack::gpu::get_type_code<refl_point>() !=
                struct_pack::gpu::get_type_code<std::array<int, 3>>());
}
"""


@pytest.mark.parametrize("cxx", ["g++", CLANG])
def test_front_end_standalone_compiles(cxx):
    """No HIP header and no reference needed: g++ 11 and clang both build a
    caller of the front end (SPK_GPU_STANDALONE: our own vocabulary types)."""
    r = _compile(cxx, USE_FRONT_END, ["-DSPK_GPU_STANDALONE"])
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.skipif(not os.path.isdir(REF_INC), reason="reference headers absent")
@pytest.mark.parametrize("cxx", ["g++", CLANG])
def test_protocol_compiles_next_to_reference(cxx):
    """struct_pack_gpu_protocol.hpp with the reference's coro_rpc headers in
    one translation unit: the GPU front end reuses the reference's errc /
    sp_config / var_int types (no redefinition), and its constexpr type
    codes equal the reference's (hash_matches_reference static_asserts)."""
    src = USE_FRONT_END.replace(
        "#include <ylt/struct_pack_gpu.hpp>",
        "#include <ylt/coro_rpc/impl/protocol/coro_rpc_protocol.hpp>\n"
        "#include <ylt/coro_rpc/impl/protocol/struct_pack_gpu_protocol.hpp>") + """
static_assert(SPK_GPU_WITH_REFERENCE);
static_assert(std::is_same_v<struct_pack::errc, decltype(struct_pack::err_code{}.ec)>);
static_assert(struct_pack::gpu::hash_matches_reference<std::vector<person>>());
static_assert(struct_pack::gpu::hash_matches_reference<refl_point>());
static_assert(struct_pack::gpu::hash_matches_reference<std::vector<with_varint>>());
void use_protocol() {
  std::tuple<std::vector<person>> args;
  (void)coro_rpc::protocol::struct_pack_gpu_protocol::deserialize_to(args, std::string_view{});
  (void)coro_rpc::protocol::struct_pack_gpu_protocol::serialize(std::get<0>(args));
  (void)coro_rpc::protocol::struct_pack_gpu_protocol::serialize(42);
}
"""
    r = _compile(cxx, src, ["-I", REF_INC, "-I", REF_INC + "/ylt/thirdparty",
                            "-I", REF_INC + "/ylt/standalone"])
    assert r.returncode == 0, r.stderr[-3000:]


OPT_IN = """
#include <ylt/struct_pack_gpu.hpp>
#include <bitset>
struct wide_rec { int32_t id; %s v; };
constexpr auto code = struct_pack::gpu::get_type_code<std::vector<wide_rec>>();
"""


@pytest.mark.parametrize("member,macro", [("wchar_t", "STRUCT_PACK_ENABLE_UNPORTABLE_TYPE"),
                                          ("std::wstring", "STRUCT_PACK_ENABLE_UNPORTABLE_TYPE"),
                                          ("std::bitset<64>", "STRUCT_PACK_ENABLE_UNPORTABLE_TYPE"),
                                          ("__int128", "STRUCT_PACK_ENABLE_INT128"),
                                          ("unsigned __int128", "STRUCT_PACK_ENABLE_INT128")])
def test_opt_in_types_need_the_reference_macros(member, macro):
    """wchar_t / std::bitset need STRUCT_PACK_ENABLE_UNPORTABLE_TYPE and the
    128-bit integers STRUCT_PACK_ENABLE_INT128, as in the reference
    (type_id.hpp:168-172,190-197,240-244,317-320): a compile error without the
    macro, a type code with it."""
    src = OPT_IN % member
    r = _compile("g++", src, ["-DSPK_GPU_STANDALONE"])
    assert r.returncode != 0 and "STRUCT_PACK_ENABLE" in r.stderr, r.stderr[-2000:]
    r = _compile("g++", src, ["-DSPK_GPU_STANDALONE", "-D" + macro])
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.skipif(not os.path.isdir(REF_INC), reason="reference headers absent")
def test_opt_in_type_codes_match_reference():
    """hash_matches_reference over the opt-in types, both front ends in one
    translation unit built with the reference's macros."""
    src = """
#include <ylt/coro_rpc/impl/protocol/coro_rpc_protocol.hpp>
#include <ylt/coro_rpc/impl/protocol/struct_pack_gpu_protocol.hpp>
#include <bitset>
struct wide_rec { int32_t id; std::u16string a; __int128 b; std::bitset<128> c; std::wstring d;
                  wchar_t e; char32_t f; unsigned __int128 g; };
static_assert(struct_pack::gpu::hash_matches_reference<std::vector<wide_rec>>());
static_assert(struct_pack::gpu::hash_matches_reference<wide_rec>());
static_assert(struct_pack::gpu::hash_matches_reference<std::u32string>());
static_assert(struct_pack::gpu::hash_matches_reference<std::bitset<64>>());
"""
    r = _compile("g++", src, ["-I", REF_INC, "-I", REF_INC + "/ylt/thirdparty",
                              "-I", REF_INC + "/ylt/standalone", "-DSTRUCT_PACK_ENABLE_INT128",
                              "-DSTRUCT_PACK_ENABLE_UNPORTABLE_TYPE"])
    assert r.returncode == 0, r.stderr[-3000:]


def test_host_walker_matches_reference_readers():
    """The front end's host walker (include/ylt/struct_pack_gpu/walk.hpp) on
    the CPU: for 27 record types, one-record and vector messages and every cut
    of them, the bytes it pulls out of the reference's memory_reader and out
    of a forward-only reader, and the bytes get_field<T, I> pulls per member,
    equal the reference's own reader positions (oracle/_ref/test_reader_field
    built next to the reference headers; no GPU call)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "test_reader_field")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/test_reader_field not built (needs /root/reference)")
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["failures"] == 0 and res["checks"] > 20000
