"""BIP68 relative lock-times against a real bcpd (regtest).

Port of the reference's test/functional/bip68-sequence.py:
* the disable flag (bit 31) turns sequence locks off; a version-2 spend with an unmet lock is
  rejected with "64: non-BIP68-final";
* 400 random version-2 spends of confirmed coins with height and time locks (MTP granularity
  512 s), each accepted or refused exactly as its locks predict;
* locks on unconfirmed (mempool) parents, across blocks mined with mocktime, a reorg that
  evicts a now-immature descendant, and re-admission after invalidateblock;
* BIP68 is not consensus before the csv deployment activates (a block holding a locked
  version-2 transaction is accepted); version-2 transactions relay on a -acceptnonstdtxn=0 node
  before and after activation (MAX_STANDARD_VERSION = 2 in this release).
"""
import os
import random
import time
from decimal import Decimal

import pytest

from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase, solve
from bitcoincashplus_amd.testing.messages import COutPoint, CTransaction, CTxIn, CTxOut, from_hex
from bitcoincashplus_amd.testing.script import CScript

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

COIN = 100000000
DISABLE_FLAG = 1 << 31
TYPE_FLAG = 1 << 22  # time-based lock
GRANULARITY = 9      # 512-second units
MASK = 0x0000FFFF
NOT_FINAL = "64: non-BIP68-final"


def hexof(tx):
    return tx.serialize().hex()


def wait_until(pred, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return
        time.sleep(0.05)
    raise AssertionError("timeout")


def send_expect(r, raw, ok):
    """sendrawtransaction; ok=False expects the non-BIP68-final reject."""
    try:
        r.sendrawtransaction(raw)
    except RPCError as e:
        assert not ok, e.message
        assert e.message == NOT_FINAL, e.message
        return False
    assert ok
    return True


@pytest.fixture
def nodes(tmp_path):
    a = BcpdProcess(str(tmp_path / "n0"), extra_args=["-gpu=0", "-blockprioritypercentage=0"])
    b = BcpdProcess(str(tmp_path / "n1"), extra_args=["-gpu=0", "-acceptnonstdtxn=0", "-blockprioritypercentage=0"])
    a.start()
    b.start()
    b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
    wait_until(lambda: a.rpc.getconnectioncount() >= 1 and b.rpc.getconnectioncount() >= 1)
    yield a, b
    a.stop()
    b.stop()


def csv_status(n):
    return n.rpc.getblockchaininfo()["bip9_softforks"]["csv"]["status"]


def test_bip68_sequence(nodes):
    n0, n1 = nodes
    r = n0.rpc
    relayfee = Decimal(str(r.getnetworkinfo()["relayfee"]))
    r.generate(110)
    # node1's coins for the version-2 relay checks, confirmed before any reorg below (node1 keeps
    # the longer branch when node0 rewinds, as in the reference)
    r.sendtoaddress(n1.rpc.getnewaddress(), 10)
    r.generate(1)
    wait_until(lambda: n1.rpc.getbestblockhash() == r.getbestblockhash(), 120)
    assert Decimal(str(n1.rpc.getbalance())) == 10
    rng = random.Random(68)

    # ---- disable flag
    r.sendtoaddress(r.getnewaddress(), 2)
    utxo = r.listunspent(0, 0)[0]
    value = int((Decimal(str(utxo["amount"])) - relayfee) * COIN)
    seq = DISABLE_FLAG | 1
    tx1 = CTransaction()
    tx1.vin = [CTxIn(COutPoint(int(utxo["txid"], 16), utxo["vout"]), nSequence=seq)]
    tx1.vout = [CTxOut(value, CScript([b"a"]))]
    tx1_id = int(r.sendrawtransaction(r.signrawtransaction(hexof(tx1), None, None, "ALL|FORKID")["hex"]), 16)
    tx2 = CTransaction()
    tx2.nVersion = 2
    tx2.vin = [CTxIn(COutPoint(tx1_id, 0), nSequence=seq & 0x7FFFFFFF)]
    tx2.vout = [CTxOut(int(value - relayfee * COIN), CScript([b"a"]))]
    send_expect(r, hexof(tx2), False)  # lock of 1 block on an unconfirmed parent
    tx2.nVersion = 1
    send_expect(r, hexof(tx2), True)  # version 1: no BIP68

    # ---- locks on confirmed inputs
    def mtp(confirmations):
        return r.getblockheader(r.getblockhash(r.getblockcount() - confirmations))["mediantime"]

    addrs = [r.getnewaddress() for _ in range(50)]
    while len(r.listunspent()) < 200:
        rng.shuffle(addrs)
        outs = {a: rng.randint(1, 20) * 0.01 for a in addrs[:rng.randint(1, 50)]}
        r.sendmany("", outs)
        r.generate(1)
    utxos = r.listunspent()
    accepted = refused = 0
    for _ in range(400):
        nin = rng.randint(1, 10)
        rng.shuffle(utxos)
        should_pass, using_locks = True, False
        tx = CTransaction()
        tx.nVersion = 2
        value = 0
        for j in range(nin):
            seq = 0xFFFFFFFE  # locks off
            if rng.randint(0, 1):
                using_locks = True
                will_pass = rng.randint(1, 10) == 1
                seq = utxos[j]["confirmations"]
                if not will_pass:
                    seq += 1
                    should_pass = False
                orig, cur = mtp(utxos[j]["confirmations"]), mtp(0)
                can_time = ((cur - orig) >> GRANULARITY) < MASK
                if rng.randint(0, 1) and can_time:
                    delta = seq << GRANULARITY
                    if will_pass and delta > cur - orig:
                        seq = (cur - orig) >> GRANULARITY
                    elif not will_pass and delta <= cur - orig:
                        seq = ((cur - orig) >> GRANULARITY) + 1
                    seq |= TYPE_FLAG
            tx.vin.append(CTxIn(COutPoint(int(utxos[j]["txid"], 16), utxos[j]["vout"]), nSequence=seq))
            value += int(Decimal(str(utxos[j]["amount"])) * COIN)
        size = len(hexof(tx)) // 2 + 120 * nin + 50
        tx.vout.append(CTxOut(int(value - relayfee * size * COIN / 1000), CScript([b"a"])))
        raw = r.signrawtransaction(hexof(tx), None, None, "ALL|FORKID")["hex"]
        if send_expect(r, raw, should_pass or not using_locks):
            accepted += 1
            utxos = r.listunspent()
        else:
            refused += 1
    assert accepted > 0 and refused > 0

    # ---- locks on unconfirmed inputs
    cur_height = r.getblockcount()
    txid = r.sendtoaddress(r.getnewaddress(), 2)
    t1 = from_hex(CTransaction(), r.getrawtransaction(txid))
    t1.rehash()
    t2 = CTransaction()
    t2.nVersion = 2
    t2.vin = [CTxIn(COutPoint(t1.sha256, 0), nSequence=0)]
    t2.vout = [CTxOut(int(t1.vout[0].nValue - relayfee * COIN), CScript([b"a"]))]
    t2 = from_hex(CTransaction(), r.signrawtransaction(hexof(t2), None, None, "ALL|FORKID")["hex"])
    t2.rehash()
    r.sendrawtransaction(hexof(t2))

    def nonzero_locks(orig, use_height):
        seq = 1 if use_height else (1 | TYPE_FLAG)
        tx = CTransaction()
        tx.nVersion = 2
        tx.vin = [CTxIn(COutPoint(orig.sha256, 0), nSequence=seq)]
        tx.vout = [CTxOut(int(orig.vout[0].nValue - relayfee * COIN), CScript([b"a"]))]
        tx.rehash()
        if send_expect(r, hexof(tx), orig.hash not in r.getrawmempool()):
            pass
        else:
            assert orig.hash in r.getrawmempool()
        return tx

    nonzero_locks(t2, True)
    nonzero_locks(t2, False)
    # keep t2 out of blocks, advance 10 blocks of mocked time
    r.prioritisetransaction(t2.hash, -1e15, int(-relayfee * COIN))
    cur_time = int(time.time())
    for _ in range(10):
        r.setmocktime(cur_time + 600)
        r.generate(1)
        cur_time += 600
    assert t2.hash in r.getrawmempool()
    nonzero_locks(t2, True)
    nonzero_locks(t2, False)
    # mine t2: a time lock of one unit on it is then satisfiable in the next block
    r.prioritisetransaction(t2.hash, 1e15, int(relayfee * COIN))
    r.setmocktime(cur_time + 600)
    r.generate(1)
    assert t2.hash not in r.getrawmempool()
    t3 = nonzero_locks(t2, False)
    assert t3.hash in r.getrawmempool()
    r.generate(1)
    assert t3.hash not in r.getrawmempool()
    t4 = nonzero_locks(t3, True)
    assert t4.hash in r.getrawmempool()
    t5 = nonzero_locks(t4, True)
    assert t5.hash not in r.getrawmempool()
    # a confirmed input beside the unconfirmed one does not lift the lock
    u = r.listunspent()[0]
    t5.vin.append(CTxIn(COutPoint(int(u["txid"], 16), u["vout"]), nSequence=1))
    t5.vout[0].nValue += int(Decimal(str(u["amount"])) * COIN)
    send_expect(r, r.signrawtransaction(hexof(t5), None, None, "ALL|FORKID")["hex"], False)
    # disconnecting the tip returns t3 and evicts t4 (its lock no longer holds)
    r.invalidateblock(r.getbestblockhash())
    assert t4.hash not in r.getrawmempool()
    assert t3.hash in r.getrawmempool()
    # two empty blocks on the fork point with old timestamps (version 3: no csv signal): the
    # reorg drops t3 (its time lock fails on the new chain) but keeps t2
    tip = int(r.getblockhash(r.getblockcount() - 1), 16)
    height = r.getblockcount()
    for _ in range(2):
        b = create_block(tip, create_coinbase(height), cur_time, height, version=3)
        solve(b)
        tip = b.sha256
        height += 1
        r.submitblock(b.serialize(legacy=True).hex(), "", True)
        cur_time += 1
    mp = r.getrawmempool()
    assert t3.hash not in mp
    assert t2.hash in mp
    r.setmocktime(0)
    r.invalidateblock(r.getblockhash(cur_height + 1))
    r.generate(10)

    # ---- BIP68 is not consensus before csv activates
    assert csv_status(n0) != "active"
    txid = r.sendtoaddress(r.getnewaddress(), 2)
    a1 = from_hex(CTransaction(), r.getrawtransaction(txid))
    a1.rehash()
    a2 = CTransaction()
    a2.nVersion = 1
    a2.vin = [CTxIn(COutPoint(a1.sha256, 0), nSequence=0)]
    a2.vout = [CTxOut(int(a1.vout[0].nValue - relayfee * COIN), CScript([b"a"]))]
    a2 = from_hex(CTransaction(), r.signrawtransaction(hexof(a2), None, None, "ALL|FORKID")["hex"])
    a2.rehash()
    r.sendrawtransaction(hexof(a2))
    a3 = CTransaction()
    a3.nVersion = 2
    a3.vin = [CTxIn(COutPoint(a2.sha256, 0), nSequence=100)]  # 100-block relative lock
    a3.vout = [CTxOut(int(a2.vout[0].nValue - relayfee * COIN), CScript([b"a"]))]
    a3.rehash()
    send_expect(r, hexof(a3), False)
    tipn = r.getblockcount()
    b = create_block(int(r.getbestblockhash(), 16), create_coinbase(tipn + 1),
                     r.getblockheader(r.getbestblockhash())["time"] + 1, tipn + 1, version=3, txs=[a1, a2, a3])
    solve(b)
    r.submitblock(b.serialize(legacy=True).hex(), "", True)
    assert r.getbestblockhash() == b.hash

    # ---- version-2 transactions are non-standard before csv, standard after
    def version2_relay():
        raw = n1.rpc.createrawtransaction([], {n1.rpc.getnewaddress(): 1.0})
        tx = from_hex(CTransaction(), n1.rpc.fundrawtransaction(raw)["hex"])
        tx.nVersion = 2
        signed = n1.rpc.signrawtransaction(hexof(tx), None, None, "ALL|FORKID")["hex"]
        try:
            n1.rpc.sendrawtransaction(signed)
            return True
        except RPCError:
            return False

    # The reference's before-activation check is vacuous (its bare `except:` also catches the
    # assert inside the `try`). What this release does: MAX_STANDARD_VERSION is 2
    # (src/primitives/transaction.h:257, policy.cpp:49) and there is no premature-version2 rule,
    # so node1 (-acceptnonstdtxn=0) relays version 2 before csv as well.
    assert version2_relay() is True
    assert r.getblockcount() < 432
    r.generate(432 - r.getblockcount())
    assert csv_status(n0) == "active"
    wait_until(lambda: n1.rpc.getbestblockhash() == r.getbestblockhash(), 120)
    assert version2_relay() is True
