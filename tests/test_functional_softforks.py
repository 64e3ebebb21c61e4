"""BIP9 deployment of CSV and the rules it switches on, over the P2P wire.

Parity:
* reference test/functional/bip9-softforks.py: the csv deployment walks DEFINED -> STARTED ->
  LOCKED_IN -> ACTIVE across 144-block regtest periods. 107 signalling blocks of a period do
  not lock in; 108 do (nRuleChangeActivationThreshold).
* reference test/functional/bip68-112-113-p2p.py: before activation, a transaction whose BIP68
  relative lock is unmet and one that is final by block time but not by median time past
  (BIP113) are valid in blocks. After activation, blocks carrying them are rejected
  ("bad-txns-nonfinal"), and a disabled relative lock (bit 31) is still fine. BIP112
  (OP_CHECKSEQUENCEVERIFY) is checked through the mempool: a spend whose nSequence is below
  the script's value is refused, and once it is high enough and the coin old enough it is
  accepted.

All of this runs below the BCP fork height. Those blocks use the legacy header and SHA-256d
proof of work.
"""
import os

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver, RejectResult
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.messages import COutPoint, CTransaction, CTxIn, CTxOut
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import OP_CHECKSEQUENCEVERIFY, OP_DROP, OP_TRUE, CScript, p2sh_script, push

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])

SIGNAL = 0x20000001  # versionbits top bits + bit 0 (csv on regtest)
NOSIGNAL = 0x20000000
PERIOD = 144
SEQUENCE_DISABLE = 1 << 31


@pytest.fixture
def node(tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-whitelist=127.0.0.1"])
    n.start()
    yield n
    n.stop()


def csv_status(n):
    return n.rpc.getblockchaininfo()["bip9_softforks"]["csv"]["status"]


class Chain:
    def __init__(self, n):
        self.n = n
        self.peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
        self.d = BlockRuleDriver(n.rpc, self.peer)
        self.B = FullBlockBuilder(n.rpc)
        self.count = 0

    def extend(self, k, version, keep=True):
        for _ in range(k):
            self.count += 1
            self.B.next_block(self.count, version=version)
            if keep:
                self.B.save_spendable_output()
            self.d.push(self.B.tip)
        self.d.wait_tip(self.B.tip.sha256)

    def height(self):
        return self.n.rpc.getblockcount()

    def tx_spending(self, out, version=1, sequence=0xFFFFFFFF, locktime=0, script=CScript([OP_TRUE])):
        B = self.B
        tx = B.create_tx(out.tx, out.n, out.tx.vout[out.n].nValue - 1000, script)
        tx.nVersion = version
        tx.vin[0].nSequence = sequence
        tx.nLockTime = locktime
        B.sign_tx(tx, out.tx, out.n)
        return tx

    def block_with(self, txs, expect=None):
        """A block on the tip holding `txs`: accepted, or rejected with reason `expect`."""
        self.count += 1
        base = self.B.tip
        self.B.next_block(self.count, version=NOSIGNAL)
        self.B.update_block(self.count, txs)
        if expect is None:
            self.d.accept(self.B.tip)
        else:
            self.d.reject(self.B.tip, RejectResult(16, expect))
            self.B.tip = base


def bip68_violator(c):
    # a relative lock of 5000 blocks on a coin that is a few hundred blocks old
    return c.tx_spending(c.B.get_spendable_output(), version=2, sequence=5000)


def bip113_violator(c):
    # final by the new block's time, not by the median time past of the last 11 blocks
    tip_time = c.B.tip.nTime
    return c.tx_spending(c.B.get_spendable_output(), version=1, sequence=0, locktime=tip_time - 1)


def test_csv_deployment_and_bip68_112_113(node):
    c = Chain(node)
    assert csv_status(node) == "defined"
    # first period without signals: the deployment starts
    c.extend(PERIOD - 1, NOSIGNAL)
    assert c.height() == PERIOD - 1
    assert csv_status(node) == "started"
    # one short of the threshold: still started
    c.extend(107, SIGNAL)
    c.extend(PERIOD - 107, NOSIGNAL)
    assert csv_status(node) == "started"
    # not enforced yet: both violators are valid in blocks
    c.block_with([bip68_violator(c)])
    c.block_with([bip113_violator(c)])
    # a period with exactly the threshold of signals locks it in
    partial = (c.height() + 1) % PERIOD  # blocks of this period already mined
    c.extend(108, SIGNAL)
    c.extend(PERIOD - 108 - partial, NOSIGNAL)
    assert (c.height() + 1) % PERIOD == 0
    assert csv_status(node) == "locked_in"
    # still not enforced while locked in
    c.block_with([bip68_violator(c)])
    c.extend(PERIOD - 1, NOSIGNAL)
    assert csv_status(node) == "active"
    info = node.rpc.getblockchaininfo()["bip9_softforks"]["csv"]
    assert info["since"] == c.height() + 1 and info["since"] % PERIOD == 0

    # ---- BIP68 / BIP113 enforced
    c.block_with([bip68_violator(c)], b"bad-txns-nonfinal")
    c.block_with([bip113_violator(c)], b"bad-txns-nonfinal")
    # a disabled relative lock, and a relative lock that is met, are fine
    c.block_with([c.tx_spending(c.B.get_spendable_output(), version=2, sequence=SEQUENCE_DISABLE | 5000)])
    c.block_with([c.tx_spending(c.B.get_spendable_output(), version=2, sequence=10)])
    # a version 1 transaction is not subject to BIP68
    c.block_with([c.tx_spending(c.B.get_spendable_output(), version=1, sequence=5000)])

    # ---- BIP112 through the mempool: a P2SH output locked by <5> OP_CHECKSEQUENCEVERIFY
    redeem = bytes(CScript([CScript.num(5), OP_CHECKSEQUENCEVERIFY, OP_DROP, OP_TRUE]))
    anyone = p2sh_script(bytes(CScript([OP_TRUE])))  # a standard output for the spends
    fund = c.tx_spending(c.B.get_spendable_output(), script=p2sh_script(redeem))
    c.block_with([fund])

    def spend(sequence):
        tx = CTransaction()
        tx.nVersion = 2
        tx.vin.append(CTxIn(COutPoint(fund.calc_sha256(), 0), bytes(push(redeem)), sequence))
        tx.vout.append(CTxOut(fund.vout[0].nValue - 10000, anyone))
        tx.rehash()
        return tx.serialize().hex()

    with pytest.raises(Exception, match="Locktime requirement not satisfied|script-verify-flag"):
        node.rpc.sendrawtransaction(spend(1))  # nSequence below the script's 5
    with pytest.raises(Exception, match="non-BIP68-final"):
        node.rpc.sendrawtransaction(spend(5))  # the coin is only one block old
    c.extend(5, NOSIGNAL, keep=False)
    txid = node.rpc.sendrawtransaction(spend(5))
    assert txid in node.rpc.getrawmempool()
    c.peer.close()
