"""Multi-node P2P functional tests over real sockets (regtest, 127.0.0.1).

Parity: reference qa/rpc-tests sendheaders.py / p2p-compactblocks.py / mempool relay
(headers-first sync, block announcement, tx relay through inv/getdata), disconnectban.py
(setban/listbanned/clearbanned/disconnectnode), nodehandling.py (addnode), and the
BCP fork transition (legacy 80-byte header chain followed by Equihash(48,5) blocks at
height >= 3000, served and validated over the wire).
"""
import os
import time

import pytest

from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


def wait_until(pred, timeout=60, step=0.1):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(step)
    raise AssertionError("wait_until timed out")


def connect(a, b):
    a.rpc.addnode(f"127.0.0.1:{b.p2p_port}", "onetry")
    wait_until(lambda: any(p["version"] for p in a.rpc.getpeerinfo()) and
               any(p["inbound"] for p in b.rpc.getpeerinfo()))


def sync_blocks(nodes, timeout=120):
    wait_until(lambda: len({n.rpc.getbestblockhash() for n in nodes}) == 1, timeout)


@pytest.fixture
def two_nodes(tmp_path):
    nodes = [BcpdProcess(str(tmp_path / f"n{i}"), extra_args=["-gpu=0"]) for i in range(2)]
    for n in nodes:
        n.start()
    yield nodes
    for n in nodes:
        n.stop()


def test_headers_sync_and_block_relay(two_nodes):
    a, b = two_nodes
    a.rpc.generate(150)
    connect(b, a)
    sync_blocks([a, b])
    assert b.rpc.getblockcount() == 150
    # new blocks are announced (headers / compact blocks) and fetched
    a.rpc.generate(3)
    sync_blocks([a, b])
    b.rpc.generate(2)
    sync_blocks([a, b])
    assert a.rpc.getblockcount() == 155
    peers = a.rpc.getpeerinfo()
    assert len(peers) == 1 and peers[0]["version"] == 70016
    assert peers[0]["subver"].startswith("/Bitcoin Cash Plus:")
    assert peers[0]["bytesrecv_per_msg"].get("headers", 0) > 0 or peers[0]["bytesrecv_per_msg"].get("cmpctblock", 0) > 0
    info = a.rpc.getnetworkinfo()
    assert info["connections"] == 1 and info["protocolversion"] == 70016
    tot = a.rpc.getnettotals()
    assert tot["totalbytessent"] > 0 and tot["totalbytesrecv"] > 0


def test_tx_relay_and_mined_by_peer(two_nodes):
    from bitcoincashplus_amd import native
    a, b = two_nodes
    connect(b, a)
    sec = bytes([9]) * 32
    wif = native.encode_secret(sec, True, "regtest")
    pub = native.ec_pubkey_create(sec, True)
    addr = native.encode_destination("pubkey", native.hash160(pub), "regtest", None)
    h = a.rpc.generatetoaddress(1, addr)[0]
    a.rpc.generate(100)
    sync_blocks([a, b])
    cb = a.rpc.getblock(h, 2)["tx"][0]
    value = cb["vout"][0]["value"]
    sats = int(round(float(value) * 1e8))
    dest = native.encode_destination("pubkey", b"\x02" * 20, "regtest", None)
    raw = a.rpc.createrawtransaction([{"txid": cb["txid"], "vout": 0}], {dest: (sats - 1000) / 1e8})
    prev = [{"txid": cb["txid"], "vout": 0, "scriptPubKey": cb["vout"][0]["scriptPubKey"]["hex"], "amount": value}]
    signed = a.rpc.signrawtransaction(raw, prev, [wif])
    txid = a.rpc.sendrawtransaction(signed["hex"])
    # relayed via inv -> getdata -> tx into the peer's mempool
    wait_until(lambda: txid in b.rpc.getrawmempool(), 60)
    # the peer mines it; the block propagates back and clears both mempools
    bh = b.rpc.generate(1)[0]
    sync_blocks([a, b])
    assert txid in a.rpc.getblock(bh)["tx"]
    wait_until(lambda: a.rpc.getrawmempool() == [] and b.rpc.getrawmempool() == [])


def test_ban_and_disconnect(two_nodes):
    a, b = two_nodes
    connect(b, a)
    assert a.rpc.getconnectioncount() == 1
    a.rpc.setban("127.0.0.1", "add", 3600)
    wait_until(lambda: a.rpc.getconnectioncount() == 0)
    banned = a.rpc.listbanned()
    assert len(banned) == 1 and banned[0]["address"] == "127.0.0.1/32"
    assert banned[0]["ban_reason"] == "manually added"
    with pytest.raises(RPCError) as e:
        a.rpc.setban("127.0.0.1", "add")
    assert e.value.code == -23
    # banned inbound connection attempts are dropped
    b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
    time.sleep(1.0)
    assert a.rpc.getconnectioncount() == 0
    a.rpc.clearbanned()
    assert a.rpc.listbanned() == []
    connect(b, a)
    peer = b.rpc.getpeerinfo()[0]
    b.rpc.disconnectnode(peer["addr"])
    wait_until(lambda: b.rpc.getconnectioncount() == 0)
    with pytest.raises(RPCError) as e:
        b.rpc.disconnectnode("127.0.0.1:1")
    assert e.value.code == -29
    # addnode bookkeeping
    b.rpc.addnode("127.0.0.1:1", "add")
    assert b.rpc.getaddednodeinfo("127.0.0.1:1")[0]["addednode"] == "127.0.0.1:1"
    with pytest.raises(RPCError):
        b.rpc.addnode("127.0.0.1:1", "add")
    b.rpc.addnode("127.0.0.1:1", "remove")
    assert b.rpc.getaddednodeinfo() == []
    assert b.rpc.setnetworkactive(False) is False
    assert b.rpc.getnetworkinfo()["networkactive"] is False
    b.rpc.setnetworkactive(True)


def test_ban_persists_across_restart(tmp_path):
    n = BcpdProcess(str(tmp_path / "bp"), extra_args=["-gpu=0"])
    n.start()
    try:
        n.rpc.setban("10.1.0.0/16", "add", 100000)
    finally:
        n.stop()
    n2 = BcpdProcess(str(tmp_path / "bp"), extra_args=["-gpu=0"], port=n.rpcport)
    n2.start()
    try:
        assert [b["address"] for b in n2.rpc.listbanned()] == ["10.1.0.0/16"]
    finally:
        n2.stop()


@pytest.mark.slow
def test_sync_across_bcp_fork(tmp_path):
    """Legacy chain to height 2999, then Equihash(48,5) blocks: a fresh peer must
    download and validate both header formats over P2P."""
    a = BcpdProcess(str(tmp_path / "fa"), extra_args=["-gpu=0"])
    b = BcpdProcess(str(tmp_path / "fb"), extra_args=["-gpu=0"])
    a.start()
    b.start()
    try:
        for _ in range(6):
            a.rpc.generate(500)
        a.rpc.generate(5)
        assert a.rpc.getblockcount() == 3005
        tip = a.rpc.getblock(a.rpc.getbestblockhash())
        assert tip["solution"] and len(tip["nonce"]) == 64
        connect(b, a)
        sync_blocks([a, b], timeout=300)
        assert b.rpc.getblockheader(b.rpc.getbestblockhash())["height"] == 3005
        a.rpc.generate(1)
        sync_blocks([a, b])
    finally:
        a.stop()
        b.stop()
