"""The node's GPU path (the shipping default when a device is visible) against a CPU twin.

Node A runs `-gpu=1 -gpusigthreshold=1`: its built-in miner solves the post-fork Equihash(48,5)
blocks on the device, ConnectBlock hands every block's signatures (the deferred CHECKSIG batch
and the speculative CHECKMULTISIG pairs) to the verify lanes, and a HEADERS message's Equihash
solutions go to the device as one batch (ProcessNewBlockHeaders -> CheckEquihashSolutions ->
GpuVerifyService::EquihashHeaders). Node B runs `-gpu=0`: every check on the CPU consensus path.

Scenario (parity anchors: reference src/validation.cpp:2011-2127 - the CCheckQueue that the
verify lanes replace - and test/functional/bcp_hardfork.py:17-30 - the regtest fork at 3000):
 1. A mines through the fork (GPU Equihash(48,5) after it); B syncs over P2P.
 2. Blocks submitted to B (submitblock, as a pool would) reach A over P2P: a fan-out block with
    1,100 P2PKH outputs and a bare 2-of-3 multisig output, then a block with 1,000 P2PKH spends
    plus the multisig spend (keys 1 and 3, so CHECKMULTISIG tries a non-matching pair).
 3. A peer sends each node a block whose 100 spends include one bad signature: both reject it
    with the same reject code and reason.
 4. A peer sends A one HEADERS message of 2,000 post-fork headers (Equihash solved here on the
    CPU); A accepts them as a headers-only branch.
Both nodes end with identical tips and `gettxoutsetinfo.hash_serialized`; A's lane counters
show the ECDSA and Equihash items the device verified, and its miner counters the GPU solves.
"""
import os
import time

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
from bitcoincashplus_amd.testing.blocktools import create_block, create_coinbase, solve
from bitcoincashplus_amd.testing.comparison import BlockRuleDriver
from bitcoincashplus_amd.testing.fullblock import FullBlockBuilder
from bitcoincashplus_amd.testing.messages import (REGTEST_BCP_HEIGHT, CBlockHeader, COutPoint, CTransaction, CTxIn,
                                                  CTxOut, hash160, msg_headers)
from bitcoincashplus_amd.testing.p2p import P2PPeer
from bitcoincashplus_amd.testing.script import (OP_0, OP_2, OP_3, OP_CHECKMULTISIG, OP_TRUE, CScript, Key,
                                                p2pkh_script, push)

pytestmark = [pytest.mark.gpu, pytest.mark.functional]

N_SPENDS = 1000
N_RESERVE = 100
FORK_MARGIN = 6  # blocks A mines past the fork height


def _ensure_binaries():
    if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
        import subprocess
        subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


def wait_until(pred, timeout=120, step=0.05, what="condition"):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return
        time.sleep(step)
    raise AssertionError(f"timed out waiting for {what}")


def lane_items(info, kind):
    return sum(L[kind] for L in info["validation_lanes"])


def _sign_p2pkh(key, tx, n_in, prev_script, value):
    sig = key.sign_input(tx, n_in, prev_script, value)
    tx.vin[n_in].scriptSig = push(sig) + push(key.pubkey)


def run_scenario(tmpdir, expect_gpu=True, log=print):
    _ensure_binaries()
    common = ["-whitelist=127.0.0.1", "-maxmempool=999", "-debug=bench"]
    a = BcpdProcess(os.path.join(tmpdir, "a"), extra_args=["-gpu=1", "-gpusigthreshold=1", *common])
    b = BcpdProcess(os.path.join(tmpdir, "b"), extra_args=["-gpu=0", *common])
    a.start()
    b.start()
    peers = []
    try:
        t0 = time.time()
        # 1. A mines through the fork; B syncs headers-first and validates the Equihash blocks on the CPU
        a.rpc.generate(REGTEST_BCP_HEIGHT - 1)
        a.rpc.generate(FORK_MARGIN)
        assert a.rpc.getblockcount() == REGTEST_BCP_HEIGHT - 1 + FORK_MARGIN
        mi = a.rpc.getmininginfo()["miner"]
        log(f"A mined {a.rpc.getblockcount()} blocks in {time.time() - t0:.1f}s; miner {mi}")
        if expect_gpu:
            assert mi["enabled"] and mi["gpu_ms"] > 0 and mi["equihash_solutions"] > 0, mi
        b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "add")
        wait_until(lambda: a.rpc.getbestblockhash() == b.rpc.getbestblockhash(), 300, what="B syncing A's chain")
        tip = b.rpc.getblockheader(b.rpc.getbestblockhash())
        assert tip["height"] >= REGTEST_BCP_HEIGHT and tip["version"] >= 4
        log(f"B synced at {time.time() - t0:.1f}s")

        # 2. blocks that enter through B reach A over P2P
        key = Key(bytes([0x42]) * 32)
        mkeys = [Key(bytes([0x51 + i]) * 32) for i in range(3)]
        pkh = p2pkh_script(hash160(key.pubkey))
        bld = FullBlockBuilder(b.rpc, key=key)

        def submit(block):
            r = b.rpc.submitblock(block.serialize().hex())
            assert r is None, r
            wait_until(lambda: a.rpc.getbestblockhash() == block.hash, 120, what=f"A reaching block {block.hash}")

        bld.next_block(0)
        funding = bld.tip.vtx[0]
        submit(bld.tip)
        for i in range(100):  # coinbase maturity
            bld.next_block(1 + i)
            submit(bld.tip)
        # fan-out: 1,100 P2PKH outputs plus a bare 2-of-3 multisig output
        value = funding.vout[0].nValue
        per = (value - 10) // (N_SPENDS + N_RESERVE + 1)
        assert per >= 1, value
        msig = CScript([OP_2, *(k.pubkey for k in mkeys), OP_3, OP_CHECKMULTISIG])
        fan = CTransaction()
        fan.vin.append(CTxIn(COutPoint(funding.calc_sha256(), 0), b"", 0xFFFFFFFF))
        for _ in range(N_SPENDS + N_RESERVE):
            fan.vout.append(CTxOut(per, pkh))
        fan.vout.append(CTxOut(per, msig))
        fan.vin[0].scriptSig = push(key.sign_input(fan, 0, funding.vout[0].scriptPubKey, value))
        fan.rehash()
        bld.next_block(200)
        bld.update_block(200, [fan])
        submit(bld.tip)

        def spend_p2pkh(i, corrupt=False):
            tx = CTransaction()
            tx.vin.append(CTxIn(COutPoint(fan.calc_sha256(), i), b"", 0xFFFFFFFF))
            tx.vout.append(CTxOut(per, CScript([OP_TRUE])))
            # a bad signature: valid DER over the digest of a different amount
            _sign_p2pkh(key, tx, 0, pkh, per + 1 if corrupt else per)
            tx.rehash()
            return tx

        gi0 = a.rpc.getgpuinfo()
        spends = [spend_p2pkh(i) for i in range(N_SPENDS)]
        ms = CTransaction()
        ms.vin.append(CTxIn(COutPoint(fan.calc_sha256(), N_SPENDS + N_RESERVE), b"", 0xFFFFFFFF))
        ms.vout.append(CTxOut(per, CScript([OP_TRUE])))
        ms.vin[0].scriptSig = bytes([OP_0]) + b"".join(push(mkeys[j].sign_input(ms, 0, msig, per)) for j in (0, 2))
        ms.rehash()
        bld.next_block(201)
        bld.update_block(201, spends + [ms])
        t1 = time.time()
        submit(bld.tip)
        log(f"{N_SPENDS}-spend block relayed and connected by A in {time.time() - t1:.2f}s")
        gi1 = a.rpc.getgpuinfo()
        log(f"A gpuinfo after the spend block: {gi1}")
        if expect_gpu:
            sv0, sv1 = gi0["sigverify"], gi1["sigverify"]
            assert gi1["enabled"] and not sv1["gpu_disabled"] and sv1["gpu_failures"] == 0, gi1
            assert sv1["gpu_sigs"] - sv0["gpu_sigs"] >= N_SPENDS, (sv0, sv1)
            assert sv1["gpu_batches"] > sv0["gpu_batches"]
            assert sv1["multisig_groups"] > sv0["multisig_groups"], (sv0, sv1)
            assert lane_items(gi1, "ecdsa_items") - lane_items(gi0, "ecdsa_items") >= N_SPENDS

        # 3. one bad signature among 100 spends: the same verdict from both nodes
        bad_spends = [spend_p2pkh(N_SPENDS + i, corrupt=(i == 57)) for i in range(N_RESERVE)]
        bld.next_block(202)
        bld.update_block(202, bad_spends)
        bad = bld.tip
        for p in a.rpc.getpeerinfo():  # keep the A-B link out of this exchange
            a.rpc.disconnectnode(p["addr"])
        wait_until(lambda: not a.rpc.getpeerinfo() and not b.rpc.getpeerinfo(), 60, what="A-B disconnect")
        rejects = []
        for n in (a, b):
            peer = P2PPeer().connect("127.0.0.1", n.p2p_port)
            peers.append(peer)
            d = BlockRuleDriver(n.rpc, peer, timeout=120)
            d.reject(bad)
            r = peer.reject_for(bad.sha256)
            assert r is not None, f"no reject message from node {'AB'[len(rejects)]}"
            rejects.append((r.code, r.reason))
        log(f"bad-signature block rejects: A {rejects[0]}  B {rejects[1]}")
        assert rejects[0] == rejects[1], rejects
        assert a.rpc.getbestblockhash() == b.rpc.getbestblockhash()

        # state parity: identical tip and UTXO set
        ua, ub = a.rpc.gettxoutsetinfo(), b.rpc.gettxoutsetinfo()
        assert ua["hash_serialized"] == ub["hash_serialized"], (ua, ub)
        assert ua["height"] == ub["height"] and ua["txouts"] == ub["txouts"]

        # 4. 2,000 post-fork headers in one HEADERS message, on top of A's tip
        tip_hash = int(a.rpc.getbestblockhash(), 16)
        tip_hdr = a.rpc.getblockheader(a.rpc.getbestblockhash())
        t2 = time.time()
        headers = []
        prev, height, ntime = tip_hash, tip_hdr["height"], tip_hdr["time"]
        for i in range(2000):
            height += 1
            ntime += 1
            blk = create_block(prev, create_coinbase(height), ntime, height)
            solve(blk)
            headers.append(CBlockHeader(blk))
            prev = blk.sha256
        log(f"2000 headers solved on the CPU in {time.time() - t2:.1f}s")
        gi2 = a.rpc.getgpuinfo()
        hp = P2PPeer().connect("127.0.0.1", a.p2p_port)
        peers.append(hp)
        t3 = time.time()
        hp.send(msg_headers(headers))
        hp.sync_with_ping(timeout=120)
        want = f"{prev:064x}"
        wait_until(lambda: any(t["hash"] == want for t in a.rpc.getchaintips()), 60, what="headers-only tip")
        log(f"A accepted 2000 headers in {time.time() - t3:.2f}s")
        tips = {t["hash"]: t for t in a.rpc.getchaintips()}
        assert tips[want]["height"] == height and tips[want]["status"] == "headers-only", tips[want]
        assert a.rpc.getbestblockhash() == f"{tip_hash:064x}"
        gi3 = a.rpc.getgpuinfo()
        if expect_gpu:
            assert lane_items(gi3, "equihash_items") - lane_items(gi2, "equihash_items") >= 2000, (gi2, gi3)
        log(f"A lanes at the end: {gi3['validation_lanes']}")
        return {"rejects": rejects, "utxo": ua["hash_serialized"], "gpuinfo": gi3}
    finally:
        for p in peers:
            try:
                p.close()
            except Exception:
                pass
        a.stop()
        b.stop()


def test_gpu_node_matches_cpu_node(tmp_path):
    run_scenario(str(tmp_path), expect_gpu=True)
