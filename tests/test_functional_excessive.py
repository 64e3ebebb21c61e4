"""Excessive block size (reference test/functional/bcp-rpc.py and bcp-cmdline.py, and the RPC
bounds of src/test/excessiveblock_tests.cpp):
get/setexcessiveblock bounds, the EB<n> comment in the user agent, and the startup checks
for -excessiveblocksize <= 1MB and -blockmaxsize above the excessive size."""
import re

import pytest

from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.node.process import BcpdProcess

pytestmark = pytest.mark.functional
ONE_MB = 1000000
LEGACY = ONE_MB
DEFAULT = 8 * ONE_MB


def test_excessiveblock_rpc(tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0"])
    n.start()
    try:
        assert n.rpc.getexcessiveblock()["excessiveBlockSize"] == DEFAULT
        assert re.match(r"/Bitcoin Cash Plus:.*\(EB8\.0.*\)/", n.rpc.getnetworkinfo()["subversion"])
        n.rpc.setexcessiveblock(LEGACY + 1)
        assert n.rpc.getexcessiveblock()["excessiveBlockSize"] == LEGACY + 1
        with pytest.raises(RPCError) as e:
            n.rpc.setexcessiveblock(LEGACY)
        assert f"Invalid parameter, excessiveblock must be larger than {LEGACY}" in str(e.value)
        assert n.rpc.getexcessiveblock()["excessiveBlockSize"] == LEGACY + 1
        for v in (2 * ONE_MB, 13 * ONE_MB, 13140000):
            n.rpc.setexcessiveblock(v)
            assert n.rpc.getexcessiveblock()["excessiveBlockSize"] == v
        assert re.match(r"/Bitcoin Cash Plus:.*\(EB13\.1.*\)/", n.rpc.getnetworkinfo()["subversion"])
    finally:
        n.stop()


def test_excessiveblocksize_cmdline(tmp_path):
    n = BcpdProcess(str(tmp_path / "a"), extra_args=["-gpu=0", f"-excessiveblocksize={2 * LEGACY}"])
    n.start()
    try:
        assert n.rpc.getexcessiveblock()["excessiveBlockSize"] == 2 * LEGACY
        assert re.match(r"/Bitcoin Cash Plus:.*\(EB2\.0.*\)/", n.rpc.getnetworkinfo()["subversion"])
    finally:
        n.stop()
    bad = BcpdProcess(str(tmp_path / "b"), extra_args=["-gpu=0", f"-excessiveblocksize={LEGACY}"])
    with pytest.raises(RuntimeError) as e:
        bad.start()
    assert "Excessive block size must be > 1,000,000 bytes (1MB)" in str(e.value)
    bad = BcpdProcess(str(tmp_path / "c"), extra_args=["-gpu=0", "-blockmaxsize=1500000",
                                                        "-excessiveblocksize=1300000"])
    with pytest.raises(RuntimeError) as e:
        bad.start()
    assert "blockmaxsize) cannot exceed the excessive block size" in str(e.value)
