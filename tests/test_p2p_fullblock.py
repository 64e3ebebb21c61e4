"""Block-rule conformance suite over the P2P wire (pure-Python peer vs a real bcpd).

Parity: reference test/functional/p2p-fullblocktest.py:147-1316 (get_tests: forks and reorgs,
coinbase value / maturity / script-size limits, sigop limits incl. CHECKMULTISIG and P2SH
counting, invalid block structures, timestamps, CVE-2012-2459 duplicate transactions, BIP30,
finality, in-block spends, subsidy, sigops after oversized pushes, mempool resurrection on
reorg, dead-branch opcodes, OP_RETURN reorgs), run with the comptool contract
(bitcoincashplus_amd/testing/comparison.py): accepted blocks become the tip; rejected
blocks do not, and the exact reject reason is asserted where the reference asserts one.

The whole sequence runs twice: before the BCP fork (80-byte headers, SHA256d PoW, the
reference's only mode) and after it (heights >= 3000 on regtest: 140-byte headers with
Equihash(48,5) solutions mined by the test itself), since the reference's Python peer could
not build post-fork blocks.
"""
import os
import random

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_coinbase, legacy_sigop_count_block, solve
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver, RejectResult
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.messages import (LEGACY_MAX_BLOCK_SIZE, MAX_BLOCK_SIGOPS_PER_MB, MAX_SCRIPT_ELEMENT_SIZE,
                                                  CBlock, COutPoint, CTransaction, CTxIn, CTxOut, ser_compact_size,
                                                  uint256_from_compact)
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import (OP_2DUP, OP_CHECKMULTISIG, OP_CHECKMULTISIGVERIFY, OP_CHECKSIG,
                                                OP_CHECKSIGVERIFY, OP_ELSE, OP_ENDIF, OP_FALSE, OP_HASH160, OP_IF,
                                                OP_INVALIDOPCODE, OP_RETURN, OP_TRUE, CScript, hash160, p2sh_script,
                                                push, signature_hash_forkid, SIGHASH_ALL, SIGHASH_FORKID)

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


@pytest.fixture
def node(tmp_path):
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-whitelist=127.0.0.1", "-debug=net"])
    n.start()
    yield n
    n.stop()


def _connect(n):
    return P2PPeer().connect("127.0.0.1", n.p2p_port)


def run_fullblock_suite(n, postfork: bool):
    if postfork:  # move the node's own chain to just below the fork: the suite mines from 3000
        n.rpc.generate(2999)
        assert n.rpc.getblockcount() == 2999
    peer = _connect(n)
    d = BlockRuleDriver(n.rpc, peer)
    B = FullBlockBuilder(n.rpc)
    block, tip, update_block = B.next_block, B.set_tip, B.update_block
    create_tx, create_and_sign_tx = B.create_tx, B.create_and_sign_tx
    save, get_out = B.save_spendable_output, B.get_spendable_output
    rej = RejectResult

    def accepted():
        d.accept(B.tip)

    def rejected(result=None):
        d.reject(B.tip, result)

    # ---- genesis of the test chain and coinbase maturity
    block(0)
    save()
    accepted()
    assert B.tip.is_new_format() == postfork
    for i in range(99):
        block(5000 + i)
        save()
        d.push(B.tip)  # sync at the end, like the reference's sync_every_block=False batch
    d.wait_tip(B.tip.sha256)
    out = [get_out() for _ in range(33)]

    # ---- forks and reorgs: b1 -> b2, b3 loses, b4 wins, b5/b6 win back
    block(1, spend=out[0]); save(); accepted()
    block(2, spend=out[1]); accepted(); save()
    tip(1); b3 = block(3, spend=out[1]); txout_b3 = (b3.vtx[1], 0)
    rejected()  # same work as b2, seen later
    block(4, spend=out[2]); accepted()
    tip(2); block(5, spend=out[2]); save(); rejected()
    block(6, spend=out[3]); accepted()

    # ---- double spend on a fork: b7 ok (less work), b8 makes it longer but double-spends
    tip(5); block(7, spend=out[2]); rejected()
    block(8, spend=out[4]); rejected()

    # ---- coinbase paying too much
    tip(6); block(9, spend=out[4], additional_coinbase_value=1)
    rejected(rej(16, b"bad-cb-amount"))
    # ... on a fork whose reorging block pays too much
    tip(5); block(10, spend=out[3]); rejected()
    block(11, spend=out[4], additional_coinbase_value=1); rejected(rej(16, b"bad-cb-amount"))

    # ---- header before block: b12 header, b13 block (stored, tip waits), b14 invalid, then b12
    tip(5); b12 = block(12, spend=out[3]); save()
    b13 = block(13, spend=out[4])
    save()
    b14 = block(14, spend=out[5], additional_coinbase_value=1)
    from bitcoincashplus_amd.testing.messages import CBlockHeader
    d.headers([CBlockHeader(b12)])
    d.push(b13)
    assert d.tip() == B.blocks[6].sha256
    d.push(b14)
    assert d.tip() == B.blocks[6].sha256
    d.push(b12)
    d.wait_tip(b13.sha256)  # b12 + b13 reorg; b14 was invalid (bad-cb-amount)
    B.tip = b13

    # ---- block sigop limit (20000 per MB): coinbase P2PK has one sigop
    lots = CScript([OP_CHECKSIG] * (MAX_BLOCK_SIGOPS_PER_MB - 1))
    tip(13); block(15, spend=out[5], script=lots); save(); accepted()
    too_many = CScript([OP_CHECKSIG] * MAX_BLOCK_SIGOPS_PER_MB)
    block(16, spend=out[6], script=too_many); rejected(rej(16, b"bad-blk-sigops"))

    # ---- spending outputs created on another fork
    tip(15); block(17, spend=txout_spend(b3)); rejected(rej(16, b"bad-txns-inputs-missingorspent"))
    tip(13); block(18, spend=txout_spend(b3)); rejected()
    block(19, spend=out[6]); rejected()

    # ---- coinbase spent too early
    tip(15); block(20, spend=out[7]); rejected(rej(16, b"bad-txns-premature-spend-of-coinbase"))
    tip(13); block(21, spend=out[6]); rejected()
    block(22, spend=out[5]); rejected()

    # ---- a block of exactly LEGACY_MAX_BLOCK_SIZE (1 MB)
    tip(15); b23 = block(23, spend=out[6])
    tx = CTransaction()
    pad = LEGACY_MAX_BLOCK_SIZE - b23.consensus_size() - 69
    tx.vout.append(CTxOut(0, CScript([b"\x00" * pad])))
    tx.vin.append(CTxIn(COutPoint(b23.vtx[1].calc_sha256(), 0)))
    b23 = update_block(23, [tx])
    assert b23.consensus_size() == LEGACY_MAX_BLOCK_SIZE
    accepted(); save()

    # ---- coinbase scriptSig length: 2..100
    tip(15); b26 = block(26, spend=out[6])
    b26.vtx[0].vin[0].scriptSig = b"\x00"
    update_block(26, []); rejected(rej(16, b"bad-cb-length"))
    block(27, spend=out[7]); rejected(rej(0, b"bad-prevblk"))
    tip(15); b28 = block(28, spend=out[6])
    b28.vtx[0].vin[0].scriptSig = b"\x00" * 101
    update_block(28, []); rejected(rej(16, b"bad-cb-length"))
    block(29, spend=out[7]); rejected(rej(0, b"bad-prevblk"))
    tip(23); b30 = block(30)
    b30.vtx[0].vin[0].scriptSig = b"\x00" * 100
    update_block(30, []); accepted(); save()

    # ---- CHECKMULTISIG(VERIFY) / CHECKSIGVERIFY sigop counting
    lots = CScript([OP_CHECKMULTISIG] * ((MAX_BLOCK_SIGOPS_PER_MB - 1) // 20) + [OP_CHECKSIG] * 19)
    block(31, spend=out[8], script=lots); save(); accepted()
    assert legacy_sigop_count_block(B.tip) == MAX_BLOCK_SIGOPS_PER_MB
    too_many = CScript([OP_CHECKMULTISIG] * (MAX_BLOCK_SIGOPS_PER_MB // 20))
    block(32, spend=out[9], script=too_many); rejected(rej(16, b"bad-blk-sigops"))
    tip(31)
    lots = CScript([OP_CHECKMULTISIGVERIFY] * ((MAX_BLOCK_SIGOPS_PER_MB - 1) // 20) + [OP_CHECKSIG] * 19)
    block(33, spend=out[9], script=lots); save(); accepted()
    too_many = CScript([OP_CHECKMULTISIGVERIFY] * (MAX_BLOCK_SIGOPS_PER_MB // 20))
    block(34, spend=out[10], script=too_many); rejected(rej(16, b"bad-blk-sigops"))
    tip(33)
    lots = CScript([OP_CHECKSIGVERIFY] * (MAX_BLOCK_SIGOPS_PER_MB - 1))
    b35 = block(35, spend=out[10], script=lots); save(); accepted()
    too_many = CScript([OP_CHECKSIGVERIFY] * MAX_BLOCK_SIGOPS_PER_MB)
    block(36, spend=out[11], script=too_many); rejected(rej(16, b"bad-blk-sigops"))

    # ---- spending a transaction of a block that failed to connect
    tip(35); b37 = block(37, spend=out[11])
    txout_b37 = (b37.vtx[1], 0)
    tx = create_and_sign_tx(out[11].tx, out[11].n, 0)
    update_block(37, [tx]); rejected(rej(16, b"bad-txns-inputs-missingorspent"))
    tip(35); block(38, spend=txout_spend(b37)); rejected(rej(16, b"bad-txns-inputs-missingorspent"))

    # ---- P2SH sigop counting: outputs whose redeem script holds 6 sigops
    tip(35); b39 = block(39)
    b39_outputs = 0
    b39_sigops_per_output = 6
    redeem = CScript([B.key.pubkey] + [OP_2DUP, OP_CHECKSIGVERIFY] * 5 + [OP_CHECKSIG])
    p2sh = p2sh_script(redeem)
    tx = create_and_sign_tx(out[11].tx, out[11].n, out[11].value, p2sh)
    tx.vout.append(CTxOut(out[11].value - 1, CScript([OP_TRUE])))  # remainder spendable by b40/b41
    tx.vout[0].nValue = 1
    B.sign_tx(tx, out[11].tx, out[11].n)
    b39 = update_block(39, [tx])
    b39_outputs += 1
    prev = tx
    target = LEGACY_MAX_BLOCK_SIZE - 1000
    size = len(b39.serialize())
    while size < target and prev.vout[1].nValue > 1:  # post-fork regtest subsidies are tiny
        t = CTransaction()
        t.vin.append(CTxIn(COutPoint(prev.calc_sha256(), 1), b"", 0xFFFFFFFF))
        t.vout.append(CTxOut(1, p2sh))
        t.vout.append(CTxOut(prev.vout[1].nValue - 1, CScript([OP_TRUE])))
        t.rehash()
        b39.vtx.append(t)
        size += len(t.serialize()) + (2 if len(b39.vtx) == 253 else 0)
        prev = t
        b39_outputs += 1
    b39 = update_block(39, [])
    accepted(); save()

    # b40: spend the P2SH outputs (6 sigops each) plus a 1-sigop first tx: over the limit by one
    tip(39); b40 = block(40, spend=out[12])
    sigops = legacy_sigop_count_block(b40)
    numTxes = (MAX_BLOCK_SIGOPS_PER_MB - sigops) // b39_sigops_per_output
    assert numTxes <= b39_outputs
    lastOutpoint = COutPoint(b40.vtx[1].calc_sha256(), 0)
    new_txs = []
    for i in range(1, numTxes + 1):
        t = CTransaction()
        t.vout.append(CTxOut(1, CScript([OP_TRUE])))
        t.vin.append(CTxIn(lastOutpoint, b""))
        t.vin.append(CTxIn(COutPoint(b39.vtx[i].calc_sha256(), 0), b""))
        sig = B.key.sign(signature_hash_forkid(redeem, t, 1, SIGHASH_ALL | SIGHASH_FORKID, 1)) + \
            bytes([SIGHASH_ALL | SIGHASH_FORKID])
        t.vin[1].scriptSig = CScript([sig, redeem])
        t.rehash()
        new_txs.append(t)
        lastOutpoint = COutPoint(t.calc_sha256(), 0)
    b40_sigops_to_fill = MAX_BLOCK_SIGOPS_PER_MB - (numTxes * b39_sigops_per_output + sigops) + 1
    t = CTransaction()
    t.vin.append(CTxIn(lastOutpoint, b""))
    t.vout.append(CTxOut(1, CScript([OP_CHECKSIG] * b40_sigops_to_fill)))
    t.rehash()
    new_txs.append(t)
    update_block(40, new_txs); rejected(rej(16, b"bad-blk-sigops"))
    # b41: the same, one sigop less: exactly at the limit
    tip(39); b41 = block(41, spend=None)
    update_block(41, b40.vtx[1:-1])
    b41_sigops_to_fill = b40_sigops_to_fill - 1
    t = CTransaction()
    t.vin.append(CTxIn(lastOutpoint, b""))
    t.vout.append(CTxOut(1, CScript([OP_CHECKSIG] * b41_sigops_to_fill)))
    t.rehash()
    update_block(41, [t]); accepted()

    # ---- constant base again: b42/b43 on b39 (b41 has the same height as b42)
    tip(39); block(42, spend=out[12]); rejected(); save()
    block(43, spend=out[13]); accepted(); save()

    # ---- really invalid blocks, built by hand
    height = B.height_of(B.tip.sha256) + 1
    coinbase = create_coinbase(height, script_pubkey=B.coinbase_script)
    b44 = CBlock(bcp_height=B.bcp_height)
    b44.nTime = B.tip.nTime + 1
    b44.hashPrevBlock = B.tip.sha256
    b44.nBits = 0x207FFFFF
    b44.nHeight = height
    b44.vtx.append(coinbase)
    b44.hashMerkleRoot = b44.calc_merkle_root()
    solve(b44)
    B.tip = b44; B.heights[b44.sha256] = height; B.blocks[44] = b44
    accepted()

    def hand_block(number, vtx, prev=None, ntime=None, nbits=0x207FFFFF, merkle=None, do_solve=True):
        p = prev or B.tip
        hh = B.height_of(p.sha256) + 1
        b = CBlock(bcp_height=B.bcp_height)
        b.nTime = (p.nTime + 1) if ntime is None else ntime
        b.hashPrevBlock = p.sha256
        b.nBits = nbits
        b.nHeight = hh
        b.vtx = list(vtx)
        b.hashMerkleRoot = b.calc_merkle_root() if merkle is None else merkle
        if do_solve:
            solve(b)
        else:
            b.rehash()
        B.tip = b; B.heights[b.sha256] = hh; B.blocks[number] = b
        return b

    # non-coinbase first transaction
    non_cb = create_tx(out[15].tx, out[15].n, 1)
    hand_block(45, [non_cb]); rejected(rej(16, b"bad-cb-missing"))
    tip(44)
    hand_block(46, [], merkle=0); rejected(rej(16, b"bad-cb-missing"))
    tip(44)
    # invalid work: a (solved-format) block whose hash exceeds the target
    b47 = block(47, solve_it=False)
    target = uint256_from_compact(b47.nBits)
    solve(b47)
    while b47.sha256 <= target:  # keep a (still valid) solution, change the nonce until the hash is too high
        b47.nNonce += 1
        if b47.is_new_format():
            from bitcoincashplus_amd import native
            st = native.EquihashState(48, 5)
            st.update(b47.equihash_input() + b47.nNonce.to_bytes(32, "little"))
            sols = native.eh_solve_cpu(48, 5, st)[0]
            if not sols:
                continue
            b47.nSolution = bytes(sols[0])
        b47.rehash()
    B.tip = b47
    rejected(rej(16, b"high-hash"))
    tip(44); b48 = block(48, solve_it=False)
    b48.nTime = int(__import__("time").time()) + 60 * 60 * 3
    B.resolve(b48); rejected(rej(16, b"time-too-new"))
    tip(44); b49 = block(49, solve_it=False)
    b49.hashMerkleRoot += 1
    B.resolve(b49); rejected(rej(16, b"bad-txnmrklroot"))
    tip(44); b50 = block(50, solve_it=False)
    b50.nBits = b50.nBits - 1
    B.resolve(b50); rejected(rej(16, b"bad-diffbits"))
    tip(44); block(51)
    cb2 = create_coinbase(51, script_pubkey=B.coinbase_script)
    update_block(51, [cb2]); rejected(rej(16, b"bad-tx-coinbase"))
    tip(44); b52 = block(52, spend=out[15])
    tx = create_tx(b52.vtx[1], 0, 1)
    update_block(52, [tx, tx]); rejected(rej(16, b"bad-txns-duplicate"))

    # ---- timestamps
    tip(43); block(53, spend=out[14]); rejected(); save()
    mtp = median_time_past(B, B.blocks[53])
    b54 = block(54, spend=out[15], solve_it=False)
    b54.nTime = mtp  # must be strictly after the median time past
    B.resolve(b54); rejected(rej(16, b"time-too-old"))
    tip(53); b55 = block(55, spend=out[15], solve_it=False)
    b55.nTime = mtp + 1
    B.resolve(b55); accepted(); save()

    # ---- CVE-2012-2459: duplicated transactions that keep the merkle root
    b57 = block(57)
    tx = create_and_sign_tx(out[16].tx, out[16].n, 1)
    tx1 = create_tx(tx, 0, 1)
    b57 = update_block(57, [tx, tx1])
    # b56: b57's header (same hash) with tx1 repeated: valid merkle root, duplicate transactions
    b56 = CBlock(b57, bcp_height=B.bcp_height)
    b56.vtx = list(b57.vtx) + [tx1]
    assert b56.calc_merkle_root() == b57.hashMerkleRoot and b56.calc_sha256() == b57.sha256
    B.tip = b56
    rejected(rej(16, b"bad-txns-duplicate"))
    tip(55); b57p2 = block("57p2")
    tx = create_and_sign_tx(out[16].tx, out[16].n, 1)
    tx1 = create_tx(tx, 0, 1); tx2 = create_tx(tx1, 0, 1); tx3 = create_tx(tx2, 0, 1); tx4 = create_tx(tx3, 0, 1)
    b57p2 = update_block("57p2", [tx, tx1, tx2, tx3, tx4])
    # b56p2: b57p2 with tx3, tx4 repeated (non-adjacent duplicates, same merkle root and hash)
    b56p2 = CBlock(b57p2, bcp_height=B.bcp_height)
    b56p2.vtx = list(b57p2.vtx) + [tx3, tx4]
    assert b56p2.calc_merkle_root() == b57p2.hashMerkleRoot
    B.tip = b56p2
    rejected(rej(16, b"bad-txns-duplicate"))
    B.tip = b57p2; accepted()
    B.tip = b57; rejected()  # 57p2 seen first
    save()

    # ---- invalid transactions
    k57p2 = "57p2"
    tip(k57p2)
    block(58, spend=out[17])
    tx = CTransaction()
    assert len(out[17].tx.vout) < 42
    tx.vin.append(CTxIn(COutPoint(out[17].tx.calc_sha256(), 42), b"", 0xFFFFFFFF))
    tx.vout.append(CTxOut(0, b""))
    update_block(58, [tx]); rejected(rej(16, b"bad-txns-inputs-missingorspent"))
    tip(k57p2); block(59)
    tx = create_and_sign_tx(out[17].tx, out[17].n, out[17].value + 1)
    update_block(59, [tx]); rejected(rej(16, b"bad-txns-in-belowout"))
    tip(k57p2); block(60, spend=out[17]); accepted(); save()

    # ---- BIP30: a coinbase identical to an unspent earlier one
    tip(60); b61 = block(61, spend=out[18])
    b61.vtx[0].vin[0].scriptSig = B.blocks[60].vtx[0].vin[0].scriptSig
    b61.vtx[0].vout = [CTxOut(o.nValue, o.scriptPubKey) for o in B.blocks[60].vtx[0].vout]
    b61.vtx[0].rehash()
    b61 = update_block(61, [])
    assert b61.vtx[0].sha256 == B.blocks[60].vtx[0].sha256
    rejected(rej(16, b"bad-txns-BIP30"))

    # ---- finality: non-final transaction and non-final coinbase
    tip(60); block(62)
    tx = CTransaction()
    tx.nLockTime = 0xFFFFFFFF
    tx.vin.append(CTxIn(COutPoint(out[18].tx.calc_sha256(), 0)))
    tx.vin[0].nSequence = 0
    tx.vout.append(CTxOut(0, CScript([OP_TRUE])))
    update_block(62, [tx]); rejected(rej(16, b"bad-txns-nonfinal"))
    tip(60); b63 = block(63)
    b63.vtx[0].nLockTime = 0xFFFFFFFF
    b63.vtx[0].vin[0].nSequence = 0xDEADBEEF
    update_block(63, []); rejected(rej(16, b"bad-txns-nonfinal"))

    # ---- a bloated (non-canonical) tx-count varint does not poison the canonical block
    tip(60); b64a = block("64a", spend=out[18])
    tx = CTransaction()
    pad = LEGACY_MAX_BLOCK_SIZE - b64a.consensus_size() - 69
    tx.vout.append(CTxOut(0, CScript([b"\x00" * pad])))
    tx.vin.append(CTxIn(COutPoint(b64a.vtx[1].calc_sha256(), 0)))
    b64a = update_block("64a", [tx])
    from bitcoincashplus_amd.testing.messages import msg_block
    bloated = b"\xff" + len(b64a.vtx).to_bytes(8, "little")
    raw = b64a.serialize(legacy=peer.legacy, tx_count_bytes=bloated)
    assert len(raw) == len(b64a.serialize(legacy=peer.legacy)) + 8
    peer.send(msg_block(raw=raw))
    peer.sync_with_ping()
    B.blocks[64] = b64a
    d.accept(b64a)
    save()

    # ---- spends inside one block
    tip(64); block(65)
    tx1 = create_and_sign_tx(out[19].tx, out[19].n, out[19].value)
    tx2 = create_and_sign_tx(tx1, 0, 0)
    update_block(65, [tx1, tx2]); accepted(); save()
    tip(65); block(66)
    tx1 = create_and_sign_tx(out[20].tx, out[20].n, out[20].value)
    tx2 = create_and_sign_tx(tx1, 0, 1)
    update_block(66, [tx2, tx1]); rejected(rej(16, b"bad-txns-inputs-missingorspent"))
    tip(65); block(67)
    tx1 = create_and_sign_tx(out[20].tx, out[20].n, out[20].value)
    tx2 = create_and_sign_tx(tx1, 0, 1)
    tx3 = create_and_sign_tx(tx1, 0, 2)
    update_block(67, [tx1, tx2, tx3]); rejected(rej(16, b"bad-txns-inputs-missingorspent"))

    # ---- subsidy + fees, exactly
    tip(65); block(68, additional_coinbase_value=10)
    tx = create_and_sign_tx(out[20].tx, out[20].n, out[20].value - 9)
    update_block(68, [tx]); rejected(rej(16, b"bad-cb-amount"))
    tip(65); block(69, additional_coinbase_value=10)
    tx = create_and_sign_tx(out[20].tx, out[20].n, out[20].value - 10)
    update_block(69, [tx]); accepted(); save()

    # ---- spending a non-existent transaction
    tip(69); block(70, spend=out[21])
    bogus = int("23c70ed7c0506e9178fc1a987f40a33946d4ad4c962b5ae3a52546da53af0c5c", 16)
    tx = CTransaction()
    tx.vin.append(CTxIn(COutPoint(bogus, 0), b"", 0xFFFFFFFF))
    tx.vout.append(CTxOut(1, b""))
    update_block(70, [tx]); rejected(rej(16, b"bad-txns-inputs-missingorspent"))

    # ---- an invalid block sharing the hash of a valid one (merkle tree trick)
    tip(69); b72 = block(72)
    tx1 = create_and_sign_tx(out[21].tx, out[21].n, 2)
    tx2 = create_and_sign_tx(tx1, 0, 1)
    b72 = update_block(72, [tx1, tx2])
    b71 = CBlock(b72, bcp_height=B.bcp_height)
    b71.vtx = list(b72.vtx) + [tx2]
    assert b71.calc_merkle_root() == b72.hashMerkleRoot
    b71.calc_sha256()
    assert b71.sha256 == b72.sha256
    B.blocks[71] = b71; B.tip = b71
    rejected(rej(16, b"bad-txns-duplicate"))
    B.tip = b72; accepted(); save()

    # ---- sigops after an oversized push are counted; inside a bad push they are not
    tip(72); b73 = block(73)
    size = MAX_BLOCK_SIGOPS_PER_MB - 1 + MAX_SCRIPT_ELEMENT_SIZE + 1 + 5 + 1
    a = bytearray([OP_CHECKSIG] * size)
    a[MAX_BLOCK_SIGOPS_PER_MB - 1] = 0x4E  # OP_PUSHDATA4
    element = MAX_SCRIPT_ELEMENT_SIZE + 1
    a[MAX_BLOCK_SIGOPS_PER_MB:MAX_BLOCK_SIGOPS_PER_MB + 4] = element.to_bytes(4, "little")
    tx = create_and_sign_tx(out[22].tx, 0, 1, CScript(bytes(a)))
    b73 = update_block(73, [tx])
    assert legacy_sigop_count_block(b73) == MAX_BLOCK_SIGOPS_PER_MB + 1
    rejected(rej(16, b"bad-blk-sigops"))
    tip(72); b74 = block(74)
    size = MAX_BLOCK_SIGOPS_PER_MB - 1 + MAX_SCRIPT_ELEMENT_SIZE + 42
    a = bytearray([OP_CHECKSIG] * size)
    a[MAX_BLOCK_SIGOPS_PER_MB] = 0x4E
    a[MAX_BLOCK_SIGOPS_PER_MB + 1:MAX_BLOCK_SIGOPS_PER_MB + 5] = b"\xfe\xff\xff\xff"
    tx = create_and_sign_tx(out[22].tx, 0, 1, CScript(bytes(a)))
    update_block(74, [tx]); rejected(rej(16, b"bad-blk-sigops"))
    tip(72); b75 = block(75)
    size = MAX_BLOCK_SIGOPS_PER_MB - 1 + MAX_SCRIPT_ELEMENT_SIZE + 42
    a = bytearray([OP_CHECKSIG] * size)
    a[MAX_BLOCK_SIGOPS_PER_MB - 1] = 0x4E
    a[MAX_BLOCK_SIGOPS_PER_MB:MAX_BLOCK_SIGOPS_PER_MB + 4] = b"\xff\xff\xff\xff"
    tx = create_and_sign_tx(out[22].tx, 0, 1, CScript(bytes(a)))
    update_block(75, [tx]); accepted(); save()
    tip(75); b76 = block(76)
    size = MAX_BLOCK_SIGOPS_PER_MB - 1 + MAX_SCRIPT_ELEMENT_SIZE + 1 + 5
    a = bytearray([OP_CHECKSIG] * size)
    a[MAX_BLOCK_SIGOPS_PER_MB - 1] = 0x4E
    a[MAX_BLOCK_SIGOPS_PER_MB:MAX_BLOCK_SIGOPS_PER_MB + 4] = (len(a) - MAX_BLOCK_SIGOPS_PER_MB - 4).to_bytes(4, "little")
    tx = create_and_sign_tx(out[23].tx, 0, 1, CScript(bytes(a)))
    update_block(76, [tx]); accepted(); save()

    # ---- transaction resurrection: txs of disconnected blocks return to the mempool
    tip(76); block(77)
    tx77 = create_and_sign_tx(out[24].tx, out[24].n, out[24].value - 1000)
    update_block(77, [tx77]); accepted(); save()
    block(78)
    tx78 = create_tx(tx77, 0, tx77.vout[0].nValue - 1000)
    update_block(78, [tx78]); accepted()
    block(79)
    tx79 = create_tx(tx78, 0, tx78.vout[0].nValue - 1000)
    update_block(79, [tx79]); accepted()
    assert n.rpc.getrawmempool() == []
    tip(77); block(80, spend=out[25]); rejected(); save()
    block(81, spend=out[26]); rejected()  # other chain is as long
    block(82, spend=out[27]); accepted()  # longer: reorg
    save()
    mem = set(n.rpc.getrawmempool())
    assert {tx78.hash, tx79.hash} <= mem, mem

    # ---- invalid opcodes in a branch that is not executed
    tip(82); block(83)
    op_codes = [OP_IF, OP_INVALIDOPCODE, OP_ELSE, OP_TRUE, OP_ENDIF]
    script = CScript(op_codes)
    tx1 = create_and_sign_tx(out[28].tx, out[28].n, out[28].value, script)
    tx2 = create_and_sign_tx(tx1, 0, 0, CScript([OP_TRUE]))
    tx2.vin[0].scriptSig = CScript([OP_FALSE])
    tx2.rehash()
    update_block(83, [tx1, tx2]); accepted(); save()

    # ---- reorgs across blocks holding OP_RETURN outputs, and spending them
    tip(83); block(84)
    tx1 = create_tx(out[29].tx, out[29].n, 0, CScript([OP_RETURN]))
    tx1.vout.append(CTxOut(0, CScript([OP_TRUE])))
    tx1.vout.append(CTxOut(0, CScript([OP_TRUE])))
    tx1.vout.append(CTxOut(0, CScript([OP_TRUE])))
    tx1.vout.append(CTxOut(0, CScript([OP_TRUE])))
    tx1.calc_sha256()
    B.sign_tx(tx1, out[29].tx, out[29].n)
    tx1.rehash()
    tx2 = create_tx(tx1, 1, 0, CScript([OP_RETURN]))
    tx2.vout.append(CTxOut(0, CScript([OP_RETURN])))
    tx3 = create_tx(tx1, 2, 0, CScript([OP_RETURN]))
    tx3.vout.append(CTxOut(0, CScript([OP_TRUE])))
    tx4 = create_tx(tx1, 3, 0, CScript([OP_TRUE]))
    tx4.vout.append(CTxOut(0, CScript([OP_RETURN])))
    tx5 = create_tx(tx1, 4, 0, CScript([OP_RETURN]))
    update_block(84, [tx1, tx2, tx3, tx4, tx5]); accepted(); save()
    tip(83); block(85, spend=out[29]); rejected()
    block(86, spend=out[30]); accepted()
    tip(84); block(87, spend=out[30]); rejected()
    save()
    block(88, spend=out[31]); accepted(); save()
    block("89a", spend=out[32])
    tx = create_tx(tx1, 0, 0, CScript([OP_TRUE]))
    update_block("89a", [tx]); rejected()

    # ---- a longer reorg back and forth (the reference uses 1088 blocks; 150 here)
    tip(88)
    LARGE = 150
    for i in range(89, 89 + LARGE):
        block(i, version=4)
        d.push(B.tip)
    d.wait_tip(B.tip.sha256)
    b_end = B.tip
    tip(88)
    for i in range(89 + LARGE, 89 + 2 * LARGE):
        block(i)
        d.push(B.tip)
    assert d.tip() == b_end.sha256  # same length: first seen stays
    block(89 + 2 * LARGE)
    accepted()
    peer.close()
    return B


def txout_spend(block):
    from bitcoincashplus_amd.testing.blocktools import SpendableOutput
    return SpendableOutput(block.vtx[1], 0)


def median_time_past(B, blk) -> int:
    times = []
    h = blk.sha256
    by_hash = {b.sha256: b for b in B.blocks.values()}
    while h in by_hash and len(times) < 11:
        times.append(by_hash[h].nTime)
        h = by_hash[h].hashPrevBlock
    times.sort()
    return times[len(times) // 2]


def test_fullblock_prefork(node):
    B = run_fullblock_suite(node, postfork=False)
    assert not B.tip.is_new_format()


@pytest.mark.slow
def test_fullblock_postfork(node):
    B = run_fullblock_suite(node, postfork=True)
    assert B.tip.is_new_format() and B.tip.nSolution
