"""End-to-end regtest chain through the C++ node (reference test/functional/bcp_hardfork.py:
mine past BCPHeight=3000 so blocks switch to the 140-byte header + Equihash(48,5),
then the chain reports the switch). The embedded node runs without P2P, so getblocktemplate
refuses it with RPC_CLIENT_P2P_DISABLED, as the reference does without g_connman
(src/rpc/mining.cpp:643-646); template contents are covered by the two-node functional tests.

Every test only assumes what the module fixture guarantees (a chain of at least 101 blocks),
so the module runs in any order and under pytest-xdist's per-test distribution."""
import pytest

from bitcoincashplus_amd.node.embedded import EmbeddedNode, RPCError


@pytest.fixture(scope="module")
def node(tmp_path_factory):
    d = tmp_path_factory.mktemp("regtest")
    n = EmbeddedNode("regtest", str(d), gpu=False)
    assert n.getblockcount() == 0
    n.generate(101)
    yield n
    n.stop()


def test_genesis(node):
    assert node.getblockhash(0) == "0f9188f13cb7b2c71f2a335e3a4fc328bf5beb436012afca590b1a11466e2206"


def test_generate_prefork(node):
    start = node.getblockcount()
    if start >= 2999:
        pytest.skip("chain already past the fork")
    hashes = node.generate(3)
    assert len(hashes) == 3
    assert node.getblockcount() == start + 3
    blk = node.getblock(hashes[-1])
    assert blk["height"] == start + 3
    assert blk["solution"] == ""
    hdr_hex = node.getblockheader(hashes[-1], False)
    assert len(hdr_hex) == 160  # legacy 80-byte header before the fork


def test_utxo_and_info(node):
    info = node.getblockchaininfo()
    assert info["chain"] == "regtest" and info["blocks"] >= 101 and info["bcpheight"] == 3000
    ts = node.gettxoutsetinfo()
    assert ts["height"] == info["blocks"] and ts["txouts"] >= 101


def test_fork_transition_equihash(node):
    if node.getblockcount() < 2999:
        node.generate(2999 - node.getblockcount())
        assert node.getblockcount() == 2999
        with pytest.raises(RPCError) as e:
            node.getblocktemplate()
        assert e.value.code == -31
    start = node.getblockcount()
    node.generate(2)
    h = node.getblockhash(3000)
    blk = node.getblock(h)
    assert blk["height"] == 3000
    assert len(blk["solution"]) > 0  # Equihash(48,5) solution present
    hdr_hex = node.getblockheader(h, False)
    assert len(hdr_hex) > 280  # 140-byte header + solution
    assert len(node.getblockheader(node.getblockhash(2999), False)) == 160  # legacy below the fork
    assert node.getblockcount() == start + 2


def test_invalidate_reconsider(node):
    tip = node.getbestblockhash()
    height = node.getblockcount()
    node.invalidateblock(tip)
    assert node.getblockcount() == height - 1
    node.reconsiderblock(tip)
    assert node.getbestblockhash() == tip


def test_rpc_errors(node):
    with pytest.raises(RPCError) as e:
        node.getblockhash(10 ** 6)
    assert e.value.code == -8
    with pytest.raises(RPCError) as e:
        node.nosuchmethod()
    assert e.value.code == -32601


def test_spend_flow(node, native):
    # coinbase to a key we control, mature it, spend it (FORKID signature), mine it
    sec = bytes([7]) * 32
    wif = native.encode_secret(sec, True, "regtest")
    pub = native.ec_pubkey_create(sec, True)
    addr = native.encode_destination("pubkey", native.hash160(pub), "regtest", None)
    h = node.generatetoaddress(1, addr)[0]
    node.generate(100)
    cb = node.getblock(h, 2)["tx"][0]
    assert cb["vout"][0]["scriptPubKey"]["addresses"] == [addr]
    value = cb["vout"][0]["value"]
    dest = native.encode_destination("pubkey", b"\x01" * 20, "regtest", None)
    sats = int(round(float(value) * 1e8))
    assert sats > 2000  # regtest subsidy halves every 150 blocks
    raw = node.createrawtransaction([{"txid": cb["txid"], "vout": 0}], {dest: (sats - 500) / 1e8})
    prev = [{"txid": cb["txid"], "vout": 0, "scriptPubKey": cb["vout"][0]["scriptPubKey"]["hex"], "amount": value}]
    signed = node.signrawtransaction(raw, prev, [wif])
    assert signed["complete"], signed
    txid = node.sendrawtransaction(signed["hex"])
    assert txid in node.getrawmempool()
    entry = node.getmempoolentry(txid)
    assert abs(float(entry["fee"]) - 0.000005) < 1e-12
    # the standard-flags re-check and sig cache are exercised; now mine it
    bh = node.generate(1)[0]
    assert txid in node.getblock(bh)["tx"]
    assert node.getrawmempool() == []
    out = node.gettxout(txid, 0)
    assert out["confirmations"] == 1
    # double spend of the same coinbase is rejected
    with pytest.raises(RPCError):
        node.sendrawtransaction(signed["hex"])


def test_submitblock_duplicate(node):
    h = node.getbestblockhash()
    raw = node.getblock(h, 0)
    assert node.submitblock(raw) == "duplicate"
