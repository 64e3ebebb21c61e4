"""More reference functional scripts ported against real bcpd processes (regtest, 127.0.0.1).

Each test names the reference script it ports and asserts that script's outputs:

* rpcnamedargs.py - named RPC arguments (``help``, ``getblockhash``/``getblock``, ``echo`` arg0..arg9)
  and the "Unknown named parameter" error;
* blockchain.py - ``gettxoutsetinfo`` over the 200-block chain (8725 coins, 200 outputs, bogosize
  17000), over the genesis-only chain after ``invalidateblock``, and unchanged after
  ``reconsiderblock``; the ``getblockheader`` fields; ``verifychain(4, 0)``;
* getchaintips.py - two halves of a split network mine 10 and 20 blocks; after the join the
  short side reports the long tip as active and its own as a 10-block "valid-fork";
* invalidateblock.py - invalidating a block of the adopted chain reorgs back to the node's own;
  invalidating lower never reorgs a node to less work;
* listtransactions.py - send / receive / send-to-self / sendmany entries with accounts and
  confirmations, and watch-only entries of an imported P2SH address only with include_watchonly;
* signrawtransactions.py - complete signing with given keys, merging partly signed copies, and
  the per-input error objects for an invalid and a missing input script;
* disablewallet.py - address validation and generatetoaddress without a wallet;
* bip65-cltv.py, bipdersig.py - nodes mining with -blockversion: on regtest the version floors
  take effect at the BIP66/BIP65 heights (1251 / 1351, reference src/chainparams.cpp:341-342),
  which is where the scripts' supermajority counts land on the reference's 200-block cached
  chain. One block before, an old-version block is still mined; from there on it is refused.

The reference's cached chain (test_framework/test_framework.py, 200 blocks with P2PK coinbases)
is rebuilt here with ``generate(200)``.
"""
import os
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


def wait_until(pred, timeout=90, step=0.05):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(step)
    raise AssertionError("wait_until timed out")


def start(tmp_path, name, *args):
    n = BcpdProcess(str(tmp_path / name), extra_args=["-gpu=0", *args])
    n.start()
    return n


def connect(a, b):
    target = f"127.0.0.1:{b.p2p_port}"

    def linked():
        return any(p["addr"] == target and not p["inbound"] and p["version"] for p in a.rpc.getpeerinfo())

    if not linked():
        a.rpc.addnode(target, "onetry")
    wait_until(linked)


def disconnect(a, b):
    target = f"127.0.0.1:{b.p2p_port}"
    a.rpc.disconnectnode(target)
    wait_until(lambda: not any(p["addr"] == target for p in a.rpc.getpeerinfo()))
    wait_until(lambda: not any(p["inbound"] for p in b.rpc.getpeerinfo()))


def sync_blocks(nodes, timeout=120):
    wait_until(lambda: len({n.rpc.getbestblockhash() for n in nodes}) == 1, timeout)


def sync_mempools(nodes, timeout=60):
    wait_until(lambda: len({tuple(sorted(n.rpc.getrawmempool())) for n in nodes}) == 1, timeout)


def _eq(got, want):
    """JSON numbers arrive as floats; the reference compares amounts as Decimals."""
    if isinstance(want, Decimal) and isinstance(got, (int, float)):
        return Decimal(str(got)) == want
    return got == want


def assert_array_result(objs, to_match, expected, should_not_find=False):
    """reference test_framework/util.py assert_array_result."""
    found = 0
    for item in objs:
        if any(not _eq(item.get(k), v) for k, v in to_match.items()):
            continue
        if should_not_find:
            raise AssertionError(f"found {item} matching {to_match}")
        for k, v in expected.items():
            assert _eq(item.get(k), v), (k, item.get(k), v, item)
        found += 1
    if not should_not_find:
        assert found > 0, f"no object matching {to_match}"


def is_hash(s, length=64):
    int(s, 16)
    return length is None or len(s) == length


@pytest.fixture(scope="module")
def chain200(tmp_path_factory):
    n = BcpdProcess(str(tmp_path_factory.mktemp("c200") / "n"), extra_args=["-gpu=0"])
    n.start()
    n.rpc.generate(200)
    yield n
    n.stop()


# ------------------------------------------------------------------ rpcnamedargs.py
def test_rpcnamedargs(chain200):
    node = chain200.rpc
    h = node.help(command="getinfo")
    assert h.startswith("getinfo\n")
    with pytest.raises(RPCError) as e:
        node.help(random="getinfo")
    assert e.value.code == -8 and "Unknown named parameter" in e.value.message
    h = node.getblockhash(height=0)
    node.getblock(blockhash=h)
    assert node.echo() == []
    assert node.echo(arg0=0, arg9=9) == [0] + [None] * 8 + [9]
    assert node.echo(arg1=1) == [None, 1]
    assert node.echo(arg9=None) == [None] * 10
    assert node.echo(arg0=0, arg3=3, arg9=9) == [0] + [None] * 2 + [3] + [None] * 5 + [9]


# ------------------------------------------------------------------ blockchain.py
def test_blockchain_txoutset_and_header(chain200):
    node = chain200.rpc
    res = node.gettxoutsetinfo()
    assert Decimal(str(res["total_amount"])) == Decimal("8725.00000000")
    assert res["transactions"] == 200
    assert res["height"] == 200
    assert res["txouts"] == 200
    assert res["bogosize"] == 17000
    assert res["bestblock"] == node.getblockhash(200)
    assert 6400 < res["disk_size"] < 64000
    assert len(res["bestblock"]) == 64 and len(res["hash_serialized"]) == 64

    b1 = node.getblockhash(1)
    node.invalidateblock(b1)
    res2 = node.gettxoutsetinfo()
    assert res2["transactions"] == 0
    assert Decimal(str(res2["total_amount"])) == 0
    assert res2["height"] == 0 and res2["txouts"] == 0 and res2["bogosize"] == 0
    assert res2["bestblock"] == node.getblockhash(0)
    assert len(res2["hash_serialized"]) == 64

    node.reconsiderblock(b1)
    res3 = node.gettxoutsetinfo()
    for k in ("total_amount", "transactions", "height", "txouts", "bogosize", "bestblock", "hash_serialized"):
        assert res[k] == res3[k], k

    with pytest.raises(RPCError):
        node.getblockheader("nonsense")
    best = node.getbestblockhash()
    header = node.getblockheader(best)
    assert header["hash"] == best
    assert header["height"] == 200
    assert header["confirmations"] == 1
    assert header["previousblockhash"] == node.getblockhash(199)
    int(header["chainwork"], 16)
    assert is_hash(header["hash"]) and is_hash(header["previousblockhash"]) and is_hash(header["merkleroot"])
    assert is_hash(header["bits"], None) and is_hash(header["nonce"], None)
    for k in ("time", "mediantime", "nonceUint32", "version"):
        assert isinstance(header[k], int), k
    int(header["versionHex"], 16)
    assert isinstance(header["difficulty"], (float, Decimal))
    assert node.verifychain(4, 0) is True


# ------------------------------------------------------------------ getchaintips.py
def test_getchaintips(tmp_path):
    a, b = start(tmp_path, "a"), start(tmp_path, "b")
    try:
        a.rpc.generate(200)
        connect(b, a)
        sync_blocks([a, b])
        tips = a.rpc.getchaintips()
        assert len(tips) == 1
        assert tips[0]["branchlen"] == 0 and tips[0]["height"] == 200 and tips[0]["status"] == "active"

        disconnect(b, a)  # split the network
        a.rpc.generate(10)
        b.rpc.generate(20)
        tips = a.rpc.getchaintips()
        assert len(tips) == 1
        short_tip = tips[0]
        assert short_tip["branchlen"] == 0 and short_tip["height"] == 210 and short_tip["status"] == "active"
        tips = b.rpc.getchaintips()
        assert len(tips) == 1
        long_tip = tips[0]
        assert long_tip["branchlen"] == 0 and long_tip["height"] == 220 and long_tip["status"] == "active"

        connect(b, a)  # join
        sync_blocks([a, b])
        tips = a.rpc.getchaintips()
        assert len(tips) == 2
        assert tips[0] == long_tip
        assert tips[1]["branchlen"] == 10
        assert tips[1]["status"] == "valid-fork"
        tips[1]["branchlen"] = 0
        tips[1]["status"] = "active"
        assert tips[1] == short_tip
    finally:
        a.stop()
        b.stop()


# ------------------------------------------------------------------ invalidateblock.py
def test_invalidateblock(tmp_path):
    n = [start(tmp_path, f"n{i}") for i in range(3)]
    try:
        n[0].rpc.generate(4)
        assert n[0].rpc.getblockcount() == 4
        besthash = n[0].rpc.getbestblockhash()
        n[1].rpc.generate(6)
        assert n[1].rpc.getblockcount() == 6

        connect(n[0], n[1])  # the reorg
        sync_blocks(n[0:2])
        assert n[0].rpc.getblockcount() == 6
        badhash = n[1].rpc.getblockhash(2)
        n[0].rpc.invalidateblock(badhash)  # back to node 0's own chain
        assert n[0].rpc.getblockcount() == 4
        assert n[0].rpc.getbestblockhash() == besthash

        connect(n[1], n[2])  # never reorg to a lower-work chain
        sync_blocks(n[1:3])
        assert n[2].rpc.getblockcount() == 6
        n[1].rpc.invalidateblock(n[1].rpc.getblockhash(5))
        assert n[1].rpc.getblockcount() == 4
        n[2].rpc.invalidateblock(n[2].rpc.getblockhash(3))
        assert n[2].rpc.getblockcount() == 2
        n[2].rpc.generate(1)
        time.sleep(2)
        assert n[2].rpc.getblockcount() == 3
        assert n[0].rpc.getblockcount() == 4
        assert n[1].rpc.getblockcount() >= 4
    finally:
        for x in n:
            x.stop()


# ------------------------------------------------------------------ listtransactions.py
def test_listtransactions(tmp_path):
    n0, n1 = start(tmp_path, "n0"), start(tmp_path, "n1")
    try:
        connect(n1, n0)
        n0.rpc.generate(101)
        sync_blocks([n0, n1])  # n1 mines on n0's tip (a block on a stale tip is reorged away)
        n1.rpc.generate(1)
        sync_blocks([n0, n1])
        n0.rpc.generate(100)
        sync_blocks([n0, n1])
        r0, r1 = n0.rpc, n1.rpc

        txid = r0.sendtoaddress(r1.getnewaddress(), 0.1)
        sync_mempools([n0, n1])
        assert_array_result(r0.listtransactions(), {"txid": txid},
                            {"category": "send", "account": "", "amount": Decimal("-0.1"), "confirmations": 0})
        assert_array_result(r1.listtransactions(), {"txid": txid},
                            {"category": "receive", "account": "", "amount": Decimal("0.1"), "confirmations": 0})
        r0.generate(1)
        sync_blocks([n0, n1])
        assert_array_result(r0.listtransactions(), {"txid": txid},
                            {"category": "send", "account": "", "amount": Decimal("-0.1"), "confirmations": 1})
        assert_array_result(r1.listtransactions(), {"txid": txid},
                            {"category": "receive", "account": "", "amount": Decimal("0.1"), "confirmations": 1})

        txid = r0.sendtoaddress(r0.getnewaddress(), 0.2)  # send to self
        assert_array_result(r0.listtransactions(), {"txid": txid, "category": "send"}, {"amount": Decimal("-0.2")})
        assert_array_result(r0.listtransactions(), {"txid": txid, "category": "receive"}, {"amount": Decimal("0.2")})

        send_to = {r0.getnewaddress(): 0.11, r1.getnewaddress(): 0.22,
                   r0.getaccountaddress("from1"): 0.33, r1.getaccountaddress("toself"): 0.44}
        txid = r1.sendmany("", send_to)
        sync_mempools([n0, n1])
        assert_array_result(r1.listtransactions(), {"category": "send", "amount": Decimal("-0.11")}, {"txid": txid})
        assert_array_result(r0.listtransactions(), {"category": "receive", "amount": Decimal("0.11")}, {"txid": txid})
        assert_array_result(r1.listtransactions(), {"category": "send", "amount": Decimal("-0.22")}, {"txid": txid})
        assert_array_result(r1.listtransactions(), {"category": "receive", "amount": Decimal("0.22")}, {"txid": txid})
        assert_array_result(r1.listtransactions(), {"category": "send", "amount": Decimal("-0.33")}, {"txid": txid})
        assert_array_result(r0.listtransactions(), {"category": "receive", "amount": Decimal("0.33")},
                            {"txid": txid, "account": "from1"})
        assert_array_result(r1.listtransactions(), {"category": "send", "amount": Decimal("-0.44")},
                            {"txid": txid, "account": ""})
        assert_array_result(r1.listtransactions(), {"category": "receive", "amount": Decimal("0.44")},
                            {"txid": txid, "account": "toself"})

        multisig = r1.createmultisig(1, [r1.getnewaddress()])
        r0.importaddress(multisig["redeemScript"], "watchonly", False, True)
        txid = r1.sendtoaddress(multisig["address"], 0.1)
        r1.generate(1)
        sync_blocks([n0, n1])
        assert len(r0.listtransactions("watchonly", 100, 0, False)) == 0
        assert_array_result(r0.listtransactions("watchonly", 100, 0, True),
                            {"category": "receive", "amount": Decimal("0.1")}, {"txid": txid, "account": "watchonly"})
    finally:
        n0.stop()
        n1.stop()


# ------------------------------------------------------------------ signrawtransactions.py
def test_signrawtransactions(tmp_path):
    n = start(tmp_path, "n")
    try:
        r = n.rpc
        priv = ["cUeKHd5orzT3mz8P9pxyREHfsWtVfgsfDjiZZBcjUBAaGk1BTj7N",
                "cVKpPfVKSJxKqVpE9awvXNWuLHCa5j5tiE7K6zbUSptFpTEtiFrA"]
        inputs = [
            {"txid": "9b907ef1e3c26fc71fe4a4b3580bc75264112f95050014157059c736f0202e71", "vout": 0,
             "amount": 3.14159, "scriptPubKey": "76a91460baa0f494b38ce3c940dea67f3804dc52d1fb9488ac"},
            {"txid": "83a4f6a6b73660e13ee6cb3c6063fa3759c50c9b7521d0536022961898f4fb02", "vout": 0,
             "amount": "123.456", "scriptPubKey": "76a914669b857c03a5ed269d5d85a1ffac9ed5d663072788ac"},
        ]
        outputs = {"mpLQjfK79b7CCV4VMJWEWAj5Mpx8Up5zxB": 0.1}
        raw = r.createrawtransaction(inputs, outputs)
        signed = r.signrawtransaction(raw, inputs, priv)
        assert signed["complete"] is True and "errors" not in signed

        # a second, inconsistent transaction appended: only the first is signed (and incompletely)
        dummy = r.createrawtransaction([inputs[0]], outputs)
        unsigned = r.signrawtransaction(raw + dummy, inputs)
        assert unsigned["complete"] is False
        # merging in the fully signed copy completes it
        signed2 = r.signrawtransaction(unsigned["hex"] + dummy + signed["hex"], inputs)
        assert signed2["complete"] is True and "errors" not in signed2

        priv1 = priv[:1]
        inputs = [
            {"txid": "9b907ef1e3c26fc71fe4a4b3580bc75264112f95050014157059c736f0202e71", "vout": 0, "amount": 0},
            {"txid": "5b8673686910442c644b1f4993d8f7753c7c8fcb5c87ee40d56eaeef25204547", "vout": 7, "amount": "1.1"},
            {"txid": "9b907ef1e3c26fc71fe4a4b3580bc75264112f95050014157059c736f0202e71", "vout": 1, "amount": 2.0},
        ]
        scripts = [
            {"txid": "9b907ef1e3c26fc71fe4a4b3580bc75264112f95050014157059c736f0202e71", "vout": 0, "amount": 0,
             "scriptPubKey": "76a91460baa0f494b38ce3c940dea67f3804dc52d1fb9488ac"},
            {"txid": "5b8673686910442c644b1f4993d8f7753c7c8fcb5c87ee40d56eaeef25204547", "vout": 7, "amount": "1.1",
             "scriptPubKey": "badbadbadbad"},
        ]
        raw = r.createrawtransaction(inputs, outputs)
        dec = r.decoderawtransaction(raw)
        for i, inp in enumerate(inputs):
            assert dec["vin"][i]["txid"] == inp["txid"] and dec["vin"][i]["vout"] == inp["vout"]
        with pytest.raises(RPCError):
            r.decoderawtransaction(raw + "00")
        res = r.signrawtransaction(raw, scripts, priv1)
        assert res["complete"] is False
        assert len(res["errors"]) == 2
        for k in ("txid", "vout", "scriptSig", "sequence", "error"):
            assert k in res["errors"][0], k
        assert res["errors"][0]["txid"] == inputs[1]["txid"] and res["errors"][0]["vout"] == inputs[1]["vout"]
        assert res["errors"][1]["txid"] == inputs[2]["txid"] and res["errors"][1]["vout"] == inputs[2]["vout"]
    finally:
        n.stop()


# ------------------------------------------------------------------ disablewallet.py
def test_disablewallet(tmp_path):
    n = start(tmp_path, "n", "-disablewallet")
    try:
        r = n.rpc
        assert r.validateaddress("3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy")["isvalid"] is False
        assert r.validateaddress("mneYUmWYsuk7kySiURxCi3AGxrAqZxLgPZ")["isvalid"] is True
        try:
            r.generatetoaddress(1, "mneYUmWYsuk7kySiURxCi3AGxrAqZxLgPZ")
        except RPCError as e:
            for bad in ("Invalid address", "ProcessNewBlock, block not accepted", "Couldn't create new block"):
                assert bad not in e.message
        with pytest.raises(RPCError) as e:
            r.generatetoaddress(1, "3J98t1WpEZ73CNmQviecrnyiWrnqRhWNLy")
        assert "Invalid address" in e.value.message
    finally:
        n.stop()


# ------------------------------------------------------------------ bip65-cltv.py / bipdersig.py
def _version_floor(tmp_path, old, new, steps):
    base = start(tmp_path, "base")
    o = start(tmp_path, "old", f"-blockversion={old}")
    w = start(tmp_path, "new", f"-blockversion={new}")
    nodes = [base, o, w]
    try:
        connect(o, base)
        connect(w, base)
        base.rpc.generate(200)  # the reference's cached chain
        sync_blocks(nodes)
        for who, count in steps:
            node = o if who == "old" else w
            for _ in range(0, count, 50):
                node.rpc.generate(min(50, count - _))
            sync_blocks(nodes)
        return nodes
    except BaseException:
        for x in nodes:
            x.stop()
        raise


@pytest.mark.parametrize("old,new,floor_height,first_old", [(2, 3, 1251, 100), (3, 4, 1351, 200)],
                         ids=["bipdersig", "bip65-cltv"])
def test_blockversion_floor(tmp_path, old, new, floor_height, first_old):
    # old-version blocks, then new-version ones up to one block below the floor height minus one
    steps = [("old", first_old), ("new", floor_height - 2 - 200 - first_old)]
    base, o, w = _version_floor(tmp_path, old, new, steps)
    try:
        assert base.rpc.getblockcount() == floor_height - 2
        o.rpc.generate(1)  # an old-version block one below the floor height: still valid
        sync_blocks([base, o, w])
        assert base.rpc.getblockcount() == floor_height - 1
        w.rpc.generate(1)
        sync_blocks([base, o, w])
        assert base.rpc.getblockcount() == floor_height
        with pytest.raises(RPCError):  # from the floor height on, an old-version block is refused
            o.rpc.generate(1)
        assert base.rpc.getblockcount() == floor_height
        assert o.rpc.getblockcount() == floor_height
        w.rpc.generate(1)
        sync_blocks([base, o, w])
        assert base.rpc.getblockcount() == floor_height + 1
        blk = base.rpc.getblock(base.rpc.getblockhash(floor_height - 1))
        assert blk["version"] == old
    finally:
        for x in (base, o, w):
            x.stop()
