"""GPU: the C++20 front end (include/ylt/struct_pack_gpu.hpp) end-to-end
through libspk_codec.so, against the reference's golden bytes:
  * tests/cpp/test_device_codec.cpp standalone (built by
    __graft_entry__.build_cpp_tests) and compiled next to the reference
    header (oracle/_ref/test_device_codec_ref: struct_pack::errc, sp_config,
    var_int*_t are then the reference's own types);
  * tests/cpp/test_reader_field.cpp (oracle/_ref/test_reader_field):
    get_field<T, I> on every fixture cut at every byte, and
    deserialize_to / get_field over the reference's memory_reader and a
    forward-only reader, against the reference in the same process;
  * tests/cpp/test_gpu_protocol.cpp (oracle/_ref/test_gpu_protocol): the
    reference's coro_rpc handler executor running batch handlers with
    struct_pack_gpu_protocol, byte-compared with the reference's
    struct_pack_protocol in the same process.
The oracle/_ref binaries are built in the dev container (they include the
reference headers) and travel to the GPU box prebuilt."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_BIN = os.path.join(ROOT, "oracle", "_ref")


def _run(exe, min_checks):
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["failures"] == 0 and res["checks"] > min_checks


def test_cpp_frontend_device_roundtrips():
    import __graft_entry__ as g
    _run(g.build_cpp_tests(), 40)


@pytest.mark.parametrize("name,min_checks", [("test_device_codec_ref", 40),
                                             ("test_gpu_protocol", 25),
                                             ("test_reader_field", 50000)])
def test_cpp_next_to_reference(name, min_checks):
    exe = os.path.join(REF_BIN, name)
    if not os.path.exists(exe):
        pytest.skip(f"{name} not built (needs /root/reference at build time)")
    _run(exe, min_checks)
