"""GPU: the C++20 front end (include/ylt/struct_pack.hpp) end-to-end through
libspk_codec.so, against the reference's golden bytes
(tests/cpp/test_device_codec.cpp, built by __graft_entry__.build())."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_frontend_device_roundtrips():
    import __graft_entry__ as g
    exe = g.build_cpp_tests()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["failures"] == 0 and res["checks"] > 40
