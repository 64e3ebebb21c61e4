"""Functional tests: real bcpd processes driven over HTTP JSON-RPC / REST / bcp-cli.

Parity: reference qa/rpc-tests (httpbasics.py, rest.py, rpcbind_test.py,
mempool_persist.py, reindex.py, multi_rpc.py) — process-level behaviour rather than
in-process calls.
"""
import base64
import http.client
import json
import os
import subprocess

import pytest

from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


@pytest.fixture
def node(tmp_path):
    n = BcpdProcess(str(tmp_path / "n0"), extra_args=["-gpu=0", "-rest"])
    n.start()
    yield n
    n.stop()


def test_rpc_basics_and_cli(node):
    assert node.rpc.getblockcount() == 0
    hashes = node.rpc.generate(5)
    assert len(hashes) == 5 and node.rpc.getbestblockhash() == hashes[-1]
    # named arguments
    hdr = node.rpc.getblockheader(blockhash=hashes[0], verbose=True)
    assert hdr["height"] == 1
    # batch request
    out = node.rpc.batch([("getblockcount", []), ("getblockhash", [2]), ("nosuchmethod", [])])
    assert out[0]["result"] == 5 and out[1]["result"] == hashes[1]
    assert out[2]["error"]["code"] == -32601
    # CLI: raw string and JSON results, named args, errors -> exit code
    r = node.cli("getblockhash", "3")
    assert r.stdout.strip() == hashes[2]
    r = node.cli("-named", "getblock", f"blockhash={hashes[4]}", "verbose=false")
    assert r.stdout.strip().startswith("0")
    r = node.cli("getblock", "00" * 32, check=False)
    assert r.returncode == 5 and "Block not found" in r.stderr


def test_http_auth_and_keepalive(node):
    conn = http.client.HTTPConnection("127.0.0.1", node.rpcport, timeout=30)
    good = "Basic " + base64.b64encode(b"rt:rtpass").decode()
    for _ in range(3):  # keep-alive: several requests on one connection
        conn.request("POST", "/", '{"method":"getblockcount","params":[],"id":1}', {"Authorization": good})
        resp = conn.getresponse()
        assert resp.status == 200
        assert json.loads(resp.read())["result"] == 0
    conn.close()
    conn = http.client.HTTPConnection("127.0.0.1", node.rpcport, timeout=30)
    bad = "Basic " + base64.b64encode(b"rt:wrong").decode()
    conn.request("POST", "/", '{"method":"getblockcount","params":[],"id":1}', {"Authorization": bad})
    assert conn.getresponse().status == 401
    conn.close()


def test_rest_endpoints(node):
    hashes = node.rpc.generate(2)
    conn = http.client.HTTPConnection("127.0.0.1", node.rpcport, timeout=30)
    conn.request("GET", "/rest/chaininfo.json")
    info = json.loads(conn.getresponse().read())
    assert info["blocks"] == 2 and info["bestblockhash"] == hashes[-1]
    conn.request("GET", f"/rest/block/{hashes[0]}.json")
    blk = json.loads(conn.getresponse().read())
    assert blk["hash"] == hashes[0]
    conn.request("GET", f"/rest/headers/2/{hashes[0]}.hex")
    hexhdrs = conn.getresponse().read().decode().strip()
    assert len(hexhdrs) == 2 * 80 * 2
    txid = blk["tx"][0]["txid"]
    conn.request("GET", f"/rest/getutxos/{txid}-0.json")
    utxos = json.loads(conn.getresponse().read())
    assert utxos["chainHeight"] == 2 and len(utxos["utxos"]) == 1
    conn.request("GET", "/rest/block/" + "00" * 32 + ".json")
    assert conn.getresponse().status == 404
    conn.close()


def test_restart_persists_chain_and_mempool(tmp_path):
    d = str(tmp_path / "p")
    n = BcpdProcess(d, extra_args=["-gpu=0"])
    n.start()
    try:
        n.rpc.generate(101)
        blk = n.rpc.getblock(n.rpc.getblockhash(1), 2)
        cb = blk["tx"][0]
        assert cb["vout"][0]["value"] > 0
        tip = n.rpc.getbestblockhash()
    finally:
        n.stop()
    n2 = BcpdProcess(d, extra_args=["-gpu=0", "-checkblocks=50", "-checklevel=4"], port=n.rpcport)
    n2.start()
    try:
        assert n2.rpc.getblockcount() == 101
        assert n2.rpc.getbestblockhash() == tip
        info = n2.rpc.gettxoutsetinfo()
        assert info["height"] == 101
    finally:
        n2.stop()


def test_reindex(tmp_path):
    d = str(tmp_path / "r")
    n = BcpdProcess(d, extra_args=["-gpu=0"])
    n.start()
    try:
        n.rpc.generate(20)
        tip = n.rpc.getbestblockhash()
    finally:
        n.stop()
    n2 = BcpdProcess(d, extra_args=["-gpu=0", "-reindex"], port=n.rpcport)
    n2.start()
    try:
        assert n2.rpc.getblockcount() == 20
        assert n2.rpc.getbestblockhash() == tip
    finally:
        n2.stop()


def test_datadir_lock(tmp_path):
    d = str(tmp_path / "l")
    n = BcpdProcess(d, extra_args=["-gpu=0"])
    n.start()
    try:
        second = subprocess.run(BcpdProcess(d, extra_args=["-gpu=0"]).args(), capture_output=True, text=True,
                                timeout=60)
        assert second.returncode != 0
        assert "lock" in second.stderr.lower()
    finally:
        n.stop()


def test_rpc_warmup_and_stop_via_cli(tmp_path):
    n = BcpdProcess(str(tmp_path / "w"), extra_args=["-gpu=0"])
    n.start()
    r = n.cli("stop")
    assert "stopping" in r.stdout
    n.proc.wait(60)
    assert n.proc.returncode == 0
    with pytest.raises((ConnectionError, OSError, RPCError)):
        n.rpc.getblockcount()


def test_safe_mode(tmp_path):
    """-testsafemode raises a warning: commands not marked okSafeMode fail with
    RPC_FORBIDDEN_BY_SAFE_MODE (-2); -disablesafemode overrides (reference warnings.cpp,
    rpc/server.cpp ObserveSafeMode)."""
    n = BcpdProcess(str(tmp_path / "sm"), extra_args=["-gpu=0", "-testsafemode"])
    n.start()
    try:
        assert "testsafemode" in n.rpc.getinfo()["errors"]
        assert "testsafemode" in n.rpc.getblockchaininfo()["warnings"]
        n.rpc.getblockcount()  # okSafeMode
        with pytest.raises(RPCError) as e:
            n.rpc.sendrawtransaction("00")
        assert e.value.code == -2 and "Safe mode" in str(e.value)
    finally:
        n.stop()
    n = BcpdProcess(str(tmp_path / "sm2"), extra_args=["-gpu=0", "-testsafemode", "-disablesafemode"])
    n.start()
    try:
        with pytest.raises(RPCError) as e:
            n.rpc.sendrawtransaction("00")
        assert e.value.code != -2
    finally:
        n.stop()


def test_fee_estimates_persist(tmp_path):
    """fee_estimates.dat is written at shutdown and read back at startup (reference
    CBlockPolicyEstimator::Write/Read); estimatepriority/estimatesmartpriority answer."""
    n = BcpdProcess(str(tmp_path / "fe"), extra_args=["-gpu=0"])
    n.start()
    n.rpc.generate(3)
    assert n.rpc.estimatepriority(2) == -1
    sp = n.rpc.estimatesmartpriority(2)
    assert sp["priority"] == -1 and sp["blocks"] >= 2
    n.stop()
    found = [os.path.join(d, f) for d, _, fs in os.walk(str(tmp_path / "fe")) for f in fs if f == "fee_estimates.dat"]
    assert found and os.path.getsize(found[0]) > 100
    n.start()
    assert n.rpc.estimatefee(2) == -1
    n.stop()


def test_bip9params_and_log_flags(tmp_path):
    """-bip9params overrides a deployment's window on regtest (reference chainparams.cpp:474);
    -logtimemicros/-logips are accepted; -bip9params is rejected off regtest."""
    n = BcpdProcess(str(tmp_path / "b9"), extra_args=["-gpu=0", "-bip9params=csv:999999999999:999999999999",
                                                        "-logtimemicros", "-logips"])
    n.start()
    try:
        n.rpc.generate(300)  # two full 144-block periods
        assert n.rpc.getblockchaininfo()["bip9_softforks"]["csv"]["status"] == "defined"
    finally:
        n.stop()
    d = BcpdProcess(str(tmp_path / "b9x"), extra_args=["-gpu=0", "-bip9params=nosuchfork:0:1"])
    with pytest.raises(RuntimeError):
        d.start()
    m = BcpdProcess(str(tmp_path / "b9y"), extra_args=["-gpu=0"])
    m.start()
    try:
        m.rpc.generate(300)  # default regtest window: csv moves past "defined"
        assert m.rpc.getblockchaininfo()["bip9_softforks"]["csv"]["status"] != "defined"
    finally:
        m.stop()
