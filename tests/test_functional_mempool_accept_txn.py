"""The mempool's per-transaction sigop limit, counted through a P2SH redeem script.

Parity: reference test/functional/mempool-accept-txn.py:175-268 (one node with -norelaypriority):
a P2SH output whose redeem script holds 6 sigops (`pubkey (2DUP CHECKSIGVERIFY)x5 CHECKSIG`) is
mined; a transaction spending it whose own output script has MAX_STANDARD_TX_SIGOPS - 6 + 1
CHECKSIGs is refused with "64: bad-txns-too-many-sigops" and leaves the mempool empty; one CHECKSIG
fewer is accepted, and once mined in the next block the mempool is empty again.
"""
import os

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.node.embedded import RPCError
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.messages import COutPoint, CTransaction, CTxIn, CTxOut
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import (OP_2DUP, OP_CHECKSIG, OP_CHECKSIGVERIFY, OP_TRUE, CScript,
                                                SIGHASH_ALL, SIGHASH_FORKID, p2sh_script, signature_hash_forkid)

pytestmark = pytest.mark.functional

MAX_STANDARD_TX_SIGOPS = 20000 // 5  # reference test_framework/cdefs.py:49

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


def test_mempool_p2sh_sigop_limit(tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-whitelist=127.0.0.1", "-norelaypriority"])
    n.start()
    try:
        peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
        d = BlockRuleDriver(n.rpc, peer)
        B = FullBlockBuilder(n.rpc)
        B.next_block(0)
        B.save_spendable_output()
        d.accept(B.tip)
        for i in range(99):  # coinbase maturity
            B.next_block(5000 + i)
            B.save_spendable_output()
            d.push(B.tip)
        d.wait_tip(B.tip.sha256)
        out = [B.get_spendable_output() for _ in range(33)]

        redeem = CScript([B.key.pubkey] + [OP_2DUP, OP_CHECKSIGVERIFY] * 5 + [OP_CHECKSIG])
        p2sh_tx = B.create_and_sign_tx(out[0].tx, out[0].n, 1, p2sh_script(redeem))
        B.next_block(1)
        B.update_block(1, [p2sh_tx])
        d.accept(B.tip)

        def spend_p2sh(output_script):
            t = CTransaction()
            t.vin.append(CTxIn(COutPoint(p2sh_tx.calc_sha256(), 0), b""))
            t.vout.append(CTxOut(1, output_script))
            sig = B.key.sign(signature_hash_forkid(redeem, t, 0, SIGHASH_ALL | SIGHASH_FORKID, 1)) + \
                bytes([SIGHASH_ALL | SIGHASH_FORKID])
            t.vin[0].scriptSig = CScript([sig, redeem])
            t.rehash()
            return t

        assert redeem.sigop_count(True) == 6
        limit = MAX_STANDARD_TX_SIGOPS - redeem.sigop_count(True)
        too_many = spend_p2sh(CScript([OP_CHECKSIG] * (limit + 1)))
        with pytest.raises(RPCError) as e:
            n.rpc.sendrawtransaction(too_many.serialize().hex())
        assert e.value.message == "64: bad-txns-too-many-sigops"
        assert set(n.rpc.getrawmempool()) == set()

        at_limit = spend_p2sh(CScript([OP_CHECKSIG] * limit))
        txid = n.rpc.sendrawtransaction(at_limit.serialize().hex())
        assert set(n.rpc.getrawmempool()) == {txid}

        B.next_block(2, spend=out[1])
        B.update_block(2, [at_limit])
        d.accept(B.tip)
        assert set(n.rpc.getrawmempool()) == set()
    finally:
        n.stop()
