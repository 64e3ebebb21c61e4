"""Reference functional scripts ported against real bcpd processes (regtest, 127.0.0.1).

Each test names the reference script it ports and asserts that script's exact outputs and
reject strings:

* decodescript.py - ``decodescript`` asm of every standard scriptSig / scriptPubKey shape and the
  sighash-type decoding of ``decoderawtransaction`` (including look-alikes that must NOT decode);
* signmessages.py - ``signmessagewithprivkey`` / ``signmessage`` / ``verifymessage``;
* rawtransactions.py - missing-input rejects, 2-of-2 / 2-of-3 multisig spends signed across
  nodes, ``getrawtransaction`` verbosity types, sequence-number range checks;
* mempool_packages.py - the verbose ancestor / descendant fields of ``getrawmempool`` /
  ``getmempoolentry`` / ``getmempoolancestors`` / ``getmempooldescendants`` and their response
  to ``prioritisetransaction``, the descendant limit, reorg re-admission;
* mempool_resurrect_test.py - transactions of invalidated blocks return to the mempool;
* disconnect_ban.py - ``setban`` / ``listbanned`` / ``clearbanned`` (persistence across restart)
  and ``disconnectnode`` by address and by node id;
* p2p-feefilter.py - a peer's BIP133 feefilter suppresses tx invs below its rate;
* p2p-mempool.py - a BIP35 ``mempool`` request disconnects when bloom filters are off;
* high_priority_transaction.py - ``-blockprioritypercentage`` reserves (or not) block space for
  high-priority free transactions;
* walletbackup.py - restore from ``backupwallet`` copies and from ``dumpwallet`` files;
* plus the RPCs no other test calls: verifychain, waitforblock(height), getdifficulty,
  getnetworkhashps, getmemoryinfo, echojson, resendwallettransactions, setaccount,
  getaccountaddress.
"""
import os
import shutil
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.messages import CTransaction, from_hex, msg_feefilter, msg_mempool
from bitcoincashplus_amd.testing.p2p import P2PPeer

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

COIN = 100000000


def wait_until(pred, timeout=60, step=0.05):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(step)
    raise AssertionError("wait_until timed out")


def start(tmp_path, name, *args, port=None):
    n = BcpdProcess(str(tmp_path / name), extra_args=["-gpu=0", *args], port=port)
    n.start()
    return n


def connect(a, b):
    """a has an outbound connection to b (opened here unless one exists), handshake done."""
    target = f"127.0.0.1:{b.p2p_port}"

    def linked():
        return any(p["addr"] == target and not p["inbound"] and p["version"] for p in a.rpc.getpeerinfo())

    if not linked():
        a.rpc.addnode(target, "onetry")
    wait_until(linked)


def sync_blocks(nodes, timeout=120):
    wait_until(lambda: len({n.rpc.getbestblockhash() for n in nodes}) == 1, timeout)


def sync_mempools(nodes, timeout=120):
    wait_until(lambda: len({tuple(sorted(n.rpc.getrawmempool())) for n in nodes}) == 1, timeout)


def raises(code, fragment, fn, *a, **kw):
    with pytest.raises(RPCError) as e:
        fn(*a, **kw)
    assert e.value.code == code, (e.value.code, e.value.message)
    assert fragment in e.value.message, e.value.message
    return e.value


@pytest.fixture(scope="module")
def solo(tmp_path_factory):
    n = BcpdProcess(str(tmp_path_factory.mktemp("solo") / "n"), extra_args=["-gpu=0"])
    n.start()
    yield n
    n.stop()


# ------------------------------------------------------------------ decodescript.py
SIG = ("304502207fa7a6d1e0ee81132a269ad84e68d695483745cde8b541e3bf630749894e342a022100c1f7ab20e13e22fb"
       "95281a870f3dcf38d782e53023ee313d741ad0cfbc0c509001")
PUB = "03b0da749730dc9b4b1f4a14d6902877a92541f5368778853d9c4a0cb7802dcfb2"
PKH = "11695b6cd891484c2d49ec5aa738ec2b2f897777"


def test_decodescript_script_sigs(solo):
    d = solo.rpc.decodescript
    push_sig, push_pub = "48" + SIG, "21" + PUB
    assert d(push_sig)["asm"] == SIG                                   # P2PK scriptSig
    assert d(push_sig + push_pub)["asm"] == f"{SIG} {PUB}"               # P2PKH scriptSig
    assert d("00" + push_sig + push_sig)["asm"] == f"0 {SIG} {SIG}"      # multisig scriptSig
    assert d("5100")["asm"] == "1 0"                                     # P2SH, empty redeemScript


def test_decodescript_script_pubkeys(solo):
    d = solo.rpc.decodescript
    push_pub, push_pkh = "21" + PUB, "14" + PKH
    assert d(push_pub + "ac")["asm"] == f"{PUB} OP_CHECKSIG"
    assert d("76a9" + push_pkh + "88ac")["asm"] == f"OP_DUP OP_HASH160 {PKH} OP_EQUALVERIFY OP_CHECKSIG"
    assert d("52" + push_pub * 3 + "53ae")["asm"] == f"2 {PUB} {PUB} {PUB} 3 OP_CHECKMULTISIG"
    assert d("a9" + push_pkh + "87")["asm"] == f"OP_HASH160 {PKH} OP_EQUAL"
    # a signature look-alike after OP_RETURN is data, never sighash-decoded
    imposter = "48" + SIG
    assert d("6a" + imposter)["asm"] == "OP_RETURN " + imposter[2:]
    # CLTV redeem script: lock until block 500000
    cltv = "63" + push_pub + "ad670320a107b17568" + push_pub + "ac"
    assert d(cltv)["asm"] == (f"OP_IF {PUB} OP_CHECKSIGVERIFY OP_ELSE 500000 OP_CHECKLOCKTIMEVERIFY OP_DROP "
                              f"OP_ENDIF {PUB} OP_CHECKSIG")
    # the P2SH address of a decoded script is reported
    assert "p2sh" in d(push_pub + "ac")


MAINNET_P2PKH_TX = (
    "0100000001696a20784a2c70143f634e95227dbdfdf0ecd51647052e70854512235f5986ca010000008a47304402207174775824bec6c27000"
    "23309a168231ec80b82c6069282f5133e6f11cbb04460220570edc55c7c5da2ca687ebd0372d3546ebc3f810516a002350cac72dfe192dfb"
    "014104d3f898e6487787910a690410b7a917ef198905c27fb9d3b0a42da12aceae0544fc7088d239d9a48f2828a15a09e84043001f27cc80"
    "d162cb95404e1210161536ffffffff0100e1f505000000001976a914eb6c6e0cdb2d256a32d97b8df1fc75d1920d9bca88ac00000000")
MULTISIG_P2SH_TX = (
    "01000000018d1f5635abd06e2c7e2ddf58dc85b3de111e4ad6e0ab51bb0dcf5e84126d927300000000fdfe0000483045022100ae3b4e589d"
    "fc9d48cb82d41008dc5fa6a86f94d5c54f9935531924602730ab8002202f88cf464414c4ed9fa11b773c5ee944f66e9b05cc1e51d97abc22"
    "ce098937ea01483045022100b44883be035600e9328a01b66c7d8439b74db64187e76b99a68f7893b701d5380220225bf286493e4c4adcf9"
    "28c40f785422572eb232f84a0b83b0dea823c3a19c75014c695221020743d44be989540d27b1b4bbbcfd17721c337cb6bc9af20eb8a32520"
    "b393532f2102c0120a1dda9e51a938d39ddd9fe0ebc45ea97e1d27a7cbd671d5431416d3dd87210213820eb3d5f509d7438c9eeecb4157b2"
    "f595105e7cd564b3cdbb9ead3da41eed53aeffffffff02611e0000000000001976a914dc863734a218bfe83ef770ee9d41a27f824a6e5688"
    "acee2a02000000000017a9142a5edea39971049a540474c6a99edf0aa4074c588700000000")


def test_decoderawtransaction_sighash_asm(solo):
    dr = solo.rpc.decoderawtransaction
    r = dr(MAINNET_P2PKH_TX)
    assert r["vin"][0]["scriptSig"]["asm"] == (
        "304402207174775824bec6c2700023309a168231ec80b82c6069282f5133e6f11cbb04460220570edc55c7c5da2ca687ebd0372d3546"
        "ebc3f810516a002350cac72dfe192dfb[ALL] 04d3f898e6487787910a690410b7a917ef198905c27fb9d3b0a42da12aceae0544fc70"
        "88d239d9a48f2828a15a09e84043001f27cc80d162cb95404e1210161536")
    r = dr(MULTISIG_P2SH_TX)
    assert r["txid"] == "8e3730608c3b0bb5df54f09076e196bc292a8e39a78e73b44b6ba08c78f5cbb0"
    assert r["vin"][0]["scriptSig"]["asm"] == (
        "0 3045022100ae3b4e589dfc9d48cb82d41008dc5fa6a86f94d5c54f9935531924602730ab8002202f88cf464414c4ed9fa11b773c5e"
        "e944f66e9b05cc1e51d97abc22ce098937ea[ALL] 3045022100b44883be035600e9328a01b66c7d8439b74db64187e76b99a68f7893b7"
        "01d5380220225bf286493e4c4adcf928c40f785422572eb232f84a0b83b0dea823c3a19c75[ALL] 5221020743d44be989540d27b1b4bb"
        "bcfd17721c337cb6bc9af20eb8a32520b393532f2102c0120a1dda9e51a938d39ddd9fe0ebc45ea97e1d27a7cbd671d5431416d3dd8721"
        "0213820eb3d5f509d7438c9eeecb4157b2f595105e7cd564b3cdbb9ead3da41eed53ae")
    assert r["vout"][0]["scriptPubKey"]["asm"] == (
        "OP_DUP OP_HASH160 dc863734a218bfe83ef770ee9d41a27f824a6e56 OP_EQUALVERIFY OP_CHECKSIG")
    assert r["vout"][1]["scriptPubKey"]["asm"] == "OP_HASH160 2a5edea39971049a540474c6a99edf0aa4074c58 OP_EQUAL"
    # an OP_RETURN crafted to pass the DER checks is not decoded as a sighash type
    crafted = (
        "01000000015ded05872fdbda629c7d3d02b194763ce3b9b1535ea884e3c8e765d42e316724020000006b48304502204c10d4064885c426"
        "38cbff3585915b322de33762598321145ba033fc796971e2022100bb153ad3baa8b757e30a2175bd32852d2e1cb9080f84d7e32fcdfd66"
        "7934ef1b012103163c0ff73511ea1743fb5b98384a2ff09dd06949488028fd819f4d83f56264efffffffff0200000000000000000b6a09"
        "30060201000201000180380100000000001976a9141cabd296e753837c086da7a45a6c2fe0d49d7b7b88ac00000000")
    assert dr(crafted)["vout"][0]["scriptPubKey"]["asm"] == "OP_RETURN 300602010002010001"
    # nor are P2PKH / P2SH hashes that look like DER signatures
    lookalike = MULTISIG_P2SH_TX.replace("dc863734a218bfe83ef770ee9d41a27f824a6e56",
                                         "3011020701010101010101020601010101010101")
    lookalike = lookalike.replace("2a5edea39971049a540474c6a99edf0aa4074c58", "3011020701010101010101020601010101010101")
    r = dr(lookalike)
    assert r["vout"][0]["scriptPubKey"]["asm"] == (
        "OP_DUP OP_HASH160 3011020701010101010101020601010101010101 OP_EQUALVERIFY OP_CHECKSIG")
    assert r["vout"][1]["scriptPubKey"]["asm"] == "OP_HASH160 3011020701010101010101020601010101010101 OP_EQUAL"
    # scriptSigs of other shapes on the first transaction's input
    tx = from_hex(CTransaction(), MULTISIG_P2SH_TX)
    push_sig = tx.vin[0].scriptSig.hex()[2:(0x48 * 2 + 4)]
    der = push_sig[2:-2]
    sig2 = der + "82"

    def asm_of(script_hex):
        tx.vin[0].scriptSig = bytes.fromhex(script_hex)
        return dr(tx.serialize().hex())["vin"][0]["scriptSig"]["asm"]

    assert asm_of(push_sig) == der + "[ALL]"
    assert asm_of("48" + sig2) == der + "[NONE|ANYONECANPAY]"
    assert asm_of("00" + push_sig + "48" + sig2) == f"0 {der}[ALL] {der}[NONE|ANYONECANPAY]"
    assert asm_of("6a143011020701010101010101020601010101010101") == (
        "OP_RETURN 3011020701010101010101020601010101010101")


# ------------------------------------------------------------------ signmessages.py
def test_signmessages(solo):
    message = "This is just a test message"
    sig = solo.rpc.signmessagewithprivkey("cUeKHd5orzT3mz8P9pxyREHfsWtVfgsfDjiZZBcjUBAaGk1BTj7N", message)
    assert solo.rpc.verifymessage("mpLQjfK79b7CCV4VMJWEWAj5Mpx8Up5zxB", sig, message)
    addr = solo.rpc.getnewaddress()
    sig = solo.rpc.signmessage(addr, message)
    assert solo.rpc.verifymessage(addr, sig, message)
    assert not solo.rpc.verifymessage(addr, sig, message + "!")


# ------------------------------------------------------------------ misc RPCs with no other test
def test_misc_rpcs(solo):
    r = solo.rpc
    assert r.echojson(1, "a", [2], {"k": True}) == [1, "a", [2], {"k": True}]
    assert r.echo("x", 3) == ["x", 3]
    base = r.getblockcount()
    r.generate(3)
    assert r.verifychain() is True
    assert r.verifychain(4, 3) is True
    assert r.getdifficulty() == pytest.approx(4.656542373906925e-10)
    hps = r.getnetworkhashps()
    assert hps >= 0
    assert r.getnetworkhashps(2, base + 2) >= 0
    mem = r.getmemoryinfo()["locked"]
    for k in ("used", "free", "total", "locked", "chunks_used", "chunks_free"):
        assert k in mem
    assert mem["used"] > 0  # wallet keys (keypool, HD master) live in the locked pool
    assert mem["total"] >= mem["used"] + mem["free"] - 64
    # waitforblockheight / waitforblock return at once for a reached target, time out otherwise
    tip = r.getbestblockhash()
    got = r.waitforblockheight(base + 3, 1000)
    assert got == {"hash": tip, "height": base + 3}
    got = r.waitforblock(tip, 1000)
    assert got["hash"] == tip
    t0 = time.time()
    got = r.waitforblockheight(base + 100, 300)
    assert got["height"] == base + 3 and time.time() - t0 >= 0.25
    # accounts: setaccount / getaccountaddress / getaccount
    a = r.getnewaddress()
    r.setaccount(a, "savings")
    assert r.getaccount(a) == "savings"
    ga = r.getaccountaddress("savings")
    assert r.getaccount(ga) == "savings"
    assert r.getaccountaddress("savings") == ga  # unused address is kept
    raises(-5, "Invalid Bitcoin address", r.setaccount, "nonsense", "x")
    # resendwallettransactions: nothing to rebroadcast on a node without peers
    assert r.resendwallettransactions() == []


# ------------------------------------------------------------------ rawtransactions.py
@pytest.fixture
def three(tmp_path):
    nodes = [start(tmp_path, f"r{i}") for i in range(3)]
    connect(nodes[1], nodes[0])
    connect(nodes[2], nodes[1])
    connect(nodes[0], nodes[2])
    yield nodes
    for n in nodes:
        n.stop()


def test_rawtransactions(three):
    n0, n1, n2 = three
    n2.rpc.generate(1)
    sync_blocks(three)
    n0.rpc.generate(101)
    sync_blocks(three)
    for amt in (1.5, 1.0, 5.0):
        n0.rpc.sendtoaddress(n2.rpc.getnewaddress(), amt)
    sync_mempools(three)
    n0.rpc.generate(5)
    sync_blocks(three)
    missing = [{"txid": "1d1d4e24ed99057e84c3f80fd8fbec79ed9e1acee37da269356ecea000000000", "vout": 1}]
    raw = n2.rpc.createrawtransaction(missing, {n0.rpc.getnewaddress(): 4.998})
    signed = n2.rpc.signrawtransaction(raw, None, None, "ALL|FORKID")
    raises(-25, "Missing inputs", n2.rpc.sendrawtransaction, signed["hex"])

    # 2-of-2 multisig of node2's keys counts in node2's balance
    a1, a2 = n2.rpc.getnewaddress(), n2.rpc.getnewaddress()
    ms = n2.rpc.addmultisigaddress(2, [n2.rpc.validateaddress(a1)["pubkey"], n2.rpc.validateaddress(a2)["pubkey"]])
    bal = Decimal(str(n2.rpc.getbalance()))
    n0.rpc.sendtoaddress(ms, 1.2)
    sync_mempools(three)
    n0.rpc.generate(1)
    sync_blocks(three)
    assert Decimal(str(n2.rpc.getbalance())) == bal + Decimal("1.2")

    # 2-of-3 across nodes: node1 holds one key, node2 two; not counted as spendable
    bal = Decimal(str(n2.rpc.getbalance()))
    b1, b2, b3 = n1.rpc.getnewaddress(), n2.rpc.getnewaddress(), n2.rpc.getnewaddress()
    ms = n2.rpc.addmultisigaddress(2, [n1.rpc.validateaddress(b1)["pubkey"], n2.rpc.validateaddress(b2)["pubkey"],
                                       n2.rpc.validateaddress(b3)["pubkey"]])
    txid = n0.rpc.sendtoaddress(ms, 2.2)
    sync_mempools(three)
    n0.rpc.generate(1)
    sync_blocks(three)
    assert Decimal(str(n2.rpc.getbalance())) == bal
    dec = n0.rpc.decoderawtransaction(n0.rpc.gettransaction(txid, True)["hex"])
    vout = next(o for o in dec["vout"] if Decimal(str(o["value"])) == Decimal("2.2"))
    bal0 = Decimal(str(n0.rpc.getbalance()))
    inputs = [{"txid": txid, "vout": vout["n"], "scriptPubKey": vout["scriptPubKey"]["hex"], "amount": vout["value"]}]
    raw = n2.rpc.createrawtransaction(inputs, {n0.rpc.getnewaddress(): 2.19})
    partial = n1.rpc.signrawtransaction(raw, inputs, None, "ALL|FORKID")
    assert partial["complete"] is False
    full = n2.rpc.signrawtransaction(raw, inputs, None, "ALL|FORKID")
    assert full["complete"] is True
    n2.rpc.sendrawtransaction(full["hex"])
    dec = n0.rpc.decoderawtransaction(full["hex"])
    sync_mempools(three)
    n0.rpc.generate(1)
    sync_blocks(three)
    assert Decimal(str(n0.rpc.getbalance())) == bal0 + Decimal("50") + Decimal("2.19")

    # getrawtransaction verbosity: 0 / False / 1 / True, and the type errors
    h = dec["hash"]
    for v in ((), (0,), (False,)):
        assert n0.rpc.getrawtransaction(h, *v) == full["hex"]
    assert n0.rpc.getrawtransaction(h, 1)["hex"] == full["hex"]
    assert n0.rpc.getrawtransaction(h, True)["hex"] == full["hex"]
    for bad in ("False", [], {}):
        raises(-3, "Invalid type", n0.rpc.getrawtransaction, h, bad)

    # sequence numbers
    def with_seq(seq):
        return [{"txid": "1d1d4e24ed99057e84c3f80fd8fbec79ed9e1acee37da269356ecea000000000", "vout": 1,
                 "sequence": seq}]

    out = {n0.rpc.getnewaddress(): 1}
    assert n0.rpc.decoderawtransaction(n0.rpc.createrawtransaction(with_seq(1000), out))["vin"][0]["sequence"] == 1000
    for bad in (-1, 4294967296):
        raises(-8, "Invalid parameter, sequence number is out of range", n0.rpc.createrawtransaction,
               with_seq(bad), out)
    got = n0.rpc.decoderawtransaction(n0.rpc.createrawtransaction(with_seq(4294967294), out))
    assert got["vin"][0]["sequence"] == 4294967294


# ------------------------------------------------------------------ mempool_resurrect_test.py
def test_mempool_resurrect(tmp_path):
    n = start(tmp_path, "m", "-checkmempool=1")
    try:
        r = n.rpc
        r.generate(110)  # blocks 1..3's coinbases mature (the reference starts on a 200-block cache)
        addr = r.getnewaddress()

        def spend(txid, amount):
            raw = r.createrawtransaction([{"txid": txid, "vout": 0}], {addr: amount})
            return r.sendrawtransaction(r.signrawtransaction(raw, None, None, "ALL|FORKID")["hex"])

        coinbase = [r.getblock(r.getblockhash(h))["tx"][0] for h in (1, 2, 3)]
        s1 = [spend(t, 49.99) for t in coinbase]
        blocks = r.generate(1)
        s2 = [spend(t, 49.98) for t in s1]
        blocks += r.generate(1)
        assert r.getrawmempool() == []
        for t in s1 + s2:
            assert r.gettransaction(t)["confirmations"] > 0
        r.invalidateblock(blocks[0])
        assert set(r.getrawmempool()) == set(s1 + s2)
        for t in s1 + s2:
            assert r.gettransaction(t)["confirmations"] == 0
        r.generate(1)
        assert r.getrawmempool() == []
        for t in s1 + s2:
            assert r.gettransaction(t)["confirmations"] > 0
    finally:
        n.stop()


# ------------------------------------------------------------------ mempool_packages.py
MAX_ANCESTORS = 25
MAX_DESCENDANTS = 25


def _chain_tx(r, parent, vout, value, fee, nout):
    send = (Decimal(str(value)) - fee) / nout
    send = send.quantize(Decimal("0.00000001"))
    outs = {r.getnewaddress(): send for _ in range(nout)}
    raw = r.createrawtransaction([{"txid": parent, "vout": vout}], outs)
    txid = r.sendrawtransaction(r.signrawtransaction(raw, None, None, "ALL|FORKID")["hex"])
    assert len(r.getrawtransaction(txid, 1)["vout"]) == nout
    return txid, send


def test_mempool_packages_verbose(tmp_path):
    n0 = start(tmp_path, "p0", "-maxorphantx=1000")
    n1 = start(tmp_path, "p1", "-maxorphantx=1000", "-limitancestorcount=5")
    try:
        connect(n1, n0)
        r = n0.rpc
        r.generate(110)  # several mature coinbases (the reference starts on a 200-block cache)
        sync_blocks([n0, n1])
        utxo = r.listunspent(10)
        txid, value = utxo[0]["txid"], Decimal(str(utxo[0]["amount"]))
        fee = Decimal("0.0001")
        chain = []
        for _ in range(MAX_ANCESTORS):
            txid, value = _chain_tx(r, txid, 0, value, fee, 1)
            chain.append(txid)
        mempool = r.getrawmempool(True)
        assert len(mempool) == MAX_ANCESTORS
        dcount, dfees, dsize = 1, Decimal(0), 0
        descendants, ancestors = [], list(chain)
        for x in reversed(chain):
            e = mempool[x]
            assert r.getmempoolentry(x) == e
            assert e["descendantcount"] == dcount
            dfees += Decimal(str(e["fee"]))
            assert Decimal(str(e["modifiedfee"])) == Decimal(str(e["fee"]))
            assert Decimal(str(e["descendantfees"])) == dfees * COIN
            dsize += e["size"]
            assert e["descendantsize"] == dsize
            dcount += 1
            assert sorted(descendants) == sorted(r.getmempooldescendants(x))
            descendants.append(x)
            ancestors.remove(x)
            assert sorted(ancestors) == sorted(r.getmempoolancestors(x))
        va = r.getmempoolancestors(chain[-1], True)
        assert len(va) == len(chain) - 1 and chain[-1] not in va
        for x, e in va.items():
            assert e == mempool[x]
        vd = r.getmempooldescendants(chain[0], True)
        assert len(vd) == len(chain) - 1 and chain[0] not in vd
        for x, e in vd.items():
            assert e == mempool[x]
        # prioritisetransaction moves ancestor / descendant fees by the delta
        r.prioritisetransaction(chain[0], 0, 1000)
        mempool = r.getrawmempool(True)
        afees = Decimal(0)
        for x in chain:
            afees += Decimal(str(mempool[x]["fee"]))
            assert Decimal(str(mempool[x]["ancestorfees"])) == afees * COIN + 1000
        r.prioritisetransaction(chain[0], 0, -1000)
        r.prioritisetransaction(chain[-1], 0, 1000)
        mempool = r.getrawmempool(True)
        dfees = Decimal(0)
        for x in reversed(chain):
            dfees += Decimal(str(mempool[x]["fee"]))
            assert Decimal(str(mempool[x]["descendantfees"])) == dfees * COIN + 1000
        # one more link exceeds the ancestor limit
        raises(-26, "too-long-mempool-chain", _chain_tx, r, txid, 0, value, fee, 1)
        # node1 (ancestor limit 5) took only the first 5
        wait_until(lambda: len(n1.rpc.getrawmempool()) == 5)
        r.generate(1)
        sync_blocks([n0, n1])
        assert r.getrawmempool() == []
        # a delta survives the reorg that re-admits the chain
        r.prioritisetransaction(chain[-1], 0, 2000)
        r.invalidateblock(r.getbestblockhash())
        n1.rpc.invalidateblock(n1.rpc.getbestblockhash())
        mempool = r.getrawmempool(True)
        dfees = Decimal(0)
        for x in reversed(chain):
            dfees += Decimal(str(mempool[x]["fee"]))
            if x == chain[-1]:
                assert Decimal(str(mempool[x]["modifiedfee"])) == Decimal(str(mempool[x]["fee"])) + Decimal("0.00002")
            assert Decimal(str(mempool[x]["descendantfees"])) == dfees * COIN + 2000
        # descendant limit: a fan-out tree of 10-output transactions
        txid, vout, value = utxo[1]["txid"], utxo[1]["vout"], Decimal(str(utxo[1]["amount"]))
        txid, sent = _chain_tx(r, txid, vout, value, fee, 10)
        parent = txid
        package = [{"txid": txid, "vout": i, "amount": sent} for i in range(10)]
        rejected_at = None
        for i in range(MAX_DESCENDANTS):
            u = package.pop(0)
            try:
                txid, sent = _chain_tx(r, u["txid"], u["vout"], u["amount"], fee, 10)
            except RPCError as e:
                assert "too-long-mempool-chain" in e.message
                rejected_at = i
                break
            package += [{"txid": txid, "vout": j, "amount": sent} for j in range(10)]
            if i == MAX_DESCENDANTS - 2:
                assert r.getrawmempool(True)[parent]["descendantcount"] == MAX_DESCENDANTS
        assert rejected_at == MAX_DESCENDANTS - 1
    finally:
        n0.stop()
        n1.stop()


# ------------------------------------------------------------------ disconnect_ban.py
def test_disconnect_ban(tmp_path):
    n0 = start(tmp_path, "b0")
    n1 = start(tmp_path, "b1")
    port1 = n1.rpcport
    try:
        connect(n1, n0)
        connect(n0, n1)
        assert len(n1.rpc.getpeerinfo()) == 2
        n1.rpc.setban("127.0.0.1", "add")
        wait_until(lambda: len(n1.rpc.getpeerinfo()) == 0)
        assert len(n1.rpc.listbanned()) == 1
        n1.rpc.clearbanned()
        assert n1.rpc.listbanned() == []
        n1.rpc.setban("127.0.0.0/24", "add")
        assert len(n1.rpc.listbanned()) == 1
        raises(-23, "IP/Subnet already banned", n1.rpc.setban, "127.0.0.1", "add")
        raises(-30, "Error: Invalid IP/Subnet", n1.rpc.setban, "127.0.0.1/42", "add")
        assert len(n1.rpc.listbanned()) == 1
        raises(-30, "Error: Unban failed", n1.rpc.setban, "127.0.0.1", "remove")
        assert len(n1.rpc.listbanned()) == 1
        n1.rpc.setban("127.0.0.0/24", "remove")
        assert n1.rpc.listbanned() == []
        n1.rpc.clearbanned()
        # persistence across a restart; a 1-second ban expires
        n1.rpc.setban("127.0.0.0/32", "add")
        n1.rpc.setban("127.0.0.0/24", "add")
        n1.rpc.setban("192.168.0.1", "add", 1)
        n1.rpc.setban("2001:4d48:ac57:400:cacf:e9ff:fe1d:9c63/19", "add", 1000)
        before = n1.rpc.listbanned()
        assert before[2]["address"] == "192.168.0.1/32"
        wait_until(lambda: len(n1.rpc.listbanned()) == 3, timeout=20)
    finally:
        n1.stop()
    n1 = BcpdProcess(n1.datadir, extra_args=["-gpu=0"], port=port1, p2p_port=n1.p2p_port)
    n1.start()
    try:
        after = n1.rpc.listbanned()
        assert after[0]["address"] == "127.0.0.0/24"
        assert after[1]["address"] == "127.0.0.0/32"
        assert "/19" in after[2]["address"]
        n1.rpc.clearbanned()
        connect(n1, n0)
        connect(n0, n1)
        # disconnectnode
        addr = n0.rpc.getpeerinfo()[0]["addr"]
        raises(-32602, "Only one of address and nodeid should be provided.", n0.rpc.disconnectnode,
               address=addr, nodeid=n0.rpc.getpeerinfo()[0]["id"])
        raises(-29, "Node not found in connected nodes", n0.rpc.disconnectnode, address="221B Baker Street")
        n0.rpc.disconnectnode(address=addr)
        wait_until(lambda: len(n0.rpc.getpeerinfo()) == 1)
        assert not [p for p in n0.rpc.getpeerinfo() if p["addr"] == addr]
        connect(n0, n1)
        connect(n1, n0)
        wait_until(lambda: len(n0.rpc.getpeerinfo()) == 2)
        assert [p for p in n0.rpc.getpeerinfo() if p["addr"] == addr] or addr.startswith("127.0.0.1")
        pid = n0.rpc.getpeerinfo()[0]["id"]
        n0.rpc.disconnectnode(nodeid=pid)
        wait_until(lambda: len(n0.rpc.getpeerinfo()) == 1)
        assert not [p for p in n0.rpc.getpeerinfo() if p["id"] == pid]
    finally:
        n0.stop()
        n1.stop()


# ------------------------------------------------------------------ p2p-feefilter.py
class InvPeer(P2PPeer):
    def __init__(self):
        super().__init__()
        self.txinvs = []

    def on_inv(self, msg):
        with self.cv:
            self.txinvs += ["%064x" % i.hash for i in msg.inv if i.type == 1]


def test_p2p_feefilter(tmp_path):
    n0 = start(tmp_path, "f0")
    n1 = start(tmp_path, "f1")
    peer = None
    try:
        connect(n1, n0)
        n1.rpc.generate(101)  # out of IBD, spendable coins on node1
        sync_blocks([n0, n1])
        n0.rpc.generate(101)
        sync_blocks([n0, n1])
        peer = InvPeer().connect("127.0.0.1", n0.p2p_port)

        def invs_match(want):
            peer.wait_for(lambda: sorted(peer.txinvs) == sorted(want), 60, "tx invs")
            with peer.cv:
                peer.txinvs = []

        n1.rpc.settxfee(Decimal("0.00020000"))
        invs_match([n1.rpc.sendtoaddress(n1.rpc.getnewaddress(), 1) for _ in range(3)])
        peer.send(msg_feefilter(15000))  # 15 sat/byte
        peer.sync_with_ping()
        invs_match([n1.rpc.sendtoaddress(n1.rpc.getnewaddress(), 1) for _ in range(3)])
        # 10 sat/byte falls below the filter: not announced
        n1.rpc.settxfee(Decimal("0.00010000"))
        low = [n1.rpc.sendtoaddress(n1.rpc.getnewaddress(), 1) for _ in range(3)]
        sync_mempools([n0, n1])
        n0.rpc.settxfee(Decimal("0.00020000"))
        invs_match([n0.rpc.sendtoaddress(n0.rpc.getnewaddress(), 1)])
        assert not set(low) & set(peer.txinvs)
        peer.send(msg_feefilter(0))
        peer.sync_with_ping()
        invs_match([n1.rpc.sendtoaddress(n1.rpc.getnewaddress(), 1) for _ in range(3)])
    finally:
        if peer:
            peer.close()
        n0.stop()
        n1.stop()


# ------------------------------------------------------------------ p2p-mempool.py
def test_p2p_mempool_request_without_bloom(tmp_path):
    n = start(tmp_path, "bm", "-peerbloomfilters=0")
    try:
        peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
        peer.send(msg_mempool())
        peer.wait_for_disconnect(timeout=20)
        wait_until(lambda: n.rpc.getpeerinfo() == [])
        peer.close()
    finally:
        n.stop()


# ------------------------------------------------------------------ high_priority_transaction.py
def _hiprio_round(r, count=150, age=250):
    """150 zero-fee one-in one-out spends of aged coins (NONE|FORKID), as the reference builds
    them with create_confirmed_utxos; returns their txids."""
    addr = r.getnewaddress()
    # coins to age: split coinbases into many small outputs, then bury them
    r.generate(101)
    utxos = []
    while len(utxos) < count:
        outs = {r.getnewaddress(): Decimal("0.5") for _ in range(60)}
        r.sendmany("", outs)
        r.generate(1)
        utxos = [u for u in r.listunspent() if Decimal(str(u["amount"])) == Decimal("0.5")]
    r.generate(age)
    utxos = [u for u in r.listunspent() if Decimal(str(u["amount"])) == Decimal("0.5")][:count]
    txids = []
    for u in utxos:
        raw = r.createrawtransaction([{"txid": u["txid"], "vout": u["vout"]}], {addr: Decimal("0.5")})
        signed = r.signrawtransaction(raw, None, None, "NONE|FORKID")
        txids.append(r.sendrawtransaction(signed["hex"], True))
    return txids


def test_high_priority_transactions(tmp_path):
    threshold = COIN * 144 / 250  # AllowFreeThreshold
    n = start(tmp_path, "hp", "-blockprioritypercentage=0", "-limitfreerelay=2")
    port = n.rpcport
    try:
        txids = _hiprio_round(n.rpc)
        size = n.rpc.getmempoolinfo()["bytes"]
        mp = n.rpc.getrawmempool(True)
        for t in txids:
            assert t in mp and mp[t]["currentpriority"] > threshold
        n.rpc.generate(1)
        assert n.rpc.getmempoolinfo()["bytes"] == size  # no priority space: nothing mined
    finally:
        n.stop()
    n = BcpdProcess(n.datadir, extra_args=["-gpu=0", "-limitfreerelay=2"], port=port)
    n.start()
    try:
        txids = _hiprio_round(n.rpc)
        mp = n.rpc.getrawmempool(True)
        for t in txids:
            assert t in mp and mp[t]["currentpriority"] > threshold
        n.rpc.generate(1)
        assert n.rpc.getmempoolinfo()["bytes"] == 0  # the default priority space takes them all
    finally:
        n.stop()


# ------------------------------------------------------------------ walletbackup.py
def test_walletbackup(tmp_path):
    args = [["-keypool=100"], ["-keypool=100"], ["-keypool=100"], []]
    nodes = [start(tmp_path, f"w{i}", *a) for i, a in enumerate(args)]
    ports = [(n.rpcport, n.p2p_port) for n in nodes]

    def link():
        for i in (0, 1, 2):
            connect(nodes[i], nodes[3])
        connect(nodes[2], nodes[0])

    import random
    rnd = random.Random(7)

    def one_round():
        a = [nodes[i].rpc.getnewaddress() for i in range(3)]
        for frm, to in ((0, 1), (0, 2), (1, 0), (1, 2), (2, 0), (2, 1)):
            if rnd.randint(1, 2) == 1:
                nodes[frm].rpc.sendtoaddress(a[to], float(Decimal(rnd.randint(1, 10)) / 10))
        sync_mempools(nodes)
        nodes[3].rpc.generate(1)
        sync_blocks(nodes)

    def restart_three():
        for i in range(3):
            nodes[i] = BcpdProcess(str(tmp_path / f"w{i}"), extra_args=["-gpu=0"], port=ports[i][0],
                                   p2p_port=ports[i][1])
            nodes[i].start()
        link()

    def stop_erase_three():
        for i in range(3):
            nodes[i].stop()
        for i in range(3):
            p = os.path.join(tmp_path / f"w{i}", "regtest", "wallet.dat")
            if os.path.isdir(p):
                shutil.rmtree(p)
            else:
                os.remove(p)
        shutil.rmtree(os.path.join(tmp_path / "w2", "regtest", "blocks"))
        shutil.rmtree(os.path.join(tmp_path / "w2", "regtest", "chainstate"))

    try:
        link()
        for i in range(3):
            nodes[i].rpc.generate(1)
            sync_blocks(nodes)
        nodes[3].rpc.generate(100)
        sync_blocks(nodes)
        assert [nodes[i].rpc.getbalance() for i in range(4)] == [50, 50, 50, 0]
        for _ in range(5):
            one_round()
        for i in range(3):
            d = str(tmp_path / f"w{i}")
            nodes[i].rpc.backupwallet(d + "/wallet.bak")
            nodes[i].rpc.dumpwallet(d + "/wallet.dump")
        for _ in range(5):
            one_round()
        nodes[3].rpc.generate(101)
        sync_blocks(nodes)
        bal = [Decimal(str(nodes[i].rpc.getbalance())) for i in range(4)]
        assert sum(bal) == 5700

        # restore from the backupwallet copies
        stop_erase_three()
        for i in range(3):
            src = str(tmp_path / f"w{i}" / "wallet.bak")
            dst = os.path.join(tmp_path / f"w{i}", "regtest", "wallet.dat")
            if os.path.isdir(src):
                shutil.copytree(src, dst)
            else:
                shutil.copyfile(src, dst)
        restart_three()
        sync_blocks(nodes)
        for i in range(3):
            wait_until(lambda: Decimal(str(nodes[i].rpc.getbalance())) == bal[i])

        # restore from the dumpwallet files into fresh wallets
        stop_erase_three()
        restart_three()
        sync_blocks(nodes)
        assert [nodes[i].rpc.getbalance() for i in range(3)] == [0, 0, 0]
        for i in range(3):
            nodes[i].rpc.importwallet(str(tmp_path / f"w{i}" / "wallet.dump"))
        sync_blocks(nodes)
        for i in range(3):
            assert Decimal(str(nodes[i].rpc.getbalance())) == bal[i]
        # backing up onto the live wallet fails
        d = str(tmp_path / "w0")
        for path in (d + "/regtest/wallet.dat", d + "/./regtest/wallet.dat", d + "/regtest/", d + "/regtest"):
            raises(-4, "backup failed", nodes[0].rpc.backupwallet, path)
    finally:
        for n in nodes:
            try:
                n.stop()
            except Exception:
                pass
