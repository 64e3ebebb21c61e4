"""Device failures in validation fall back to the CPU instead of stalling sync.

BatchVerifySignatures (ConnectBlock's ECDSA batch) and CheckEquihashSolutions (header
batches) re-run a batch on the CPU when the GPU path throws, as a failed hipMalloc, launch
or device fault would, and turn the GPU path off after three consecutive failures.
`-gpufaultinjection` / `set_gpu_fault_injection` makes every such GPU batch throw, so the
fallback runs on any host. The reference has no GPU path; its CPU results are the oracle
(CPubKey::Verify, reference src/pubkey.cpp:170-193; Equihash IsValidSolution,
src/crypto/equihash.cpp:725).
"""
import os
import time

import pytest

from test_ecdsa_batch import make_items
from test_equihash import header_input


@pytest.fixture
def injected(native):
    old = native.get_gpu_sig_threshold()
    native.set_gpu_sig_threshold(1)
    native.reset_gpu_sig_failures()
    native.set_gpu_fault_injection(True)
    yield native
    native.set_gpu_fault_injection(False)
    native.reset_gpu_sig_failures()
    native.set_gpu_sig_threshold(old)


def test_sig_batch_falls_back_to_cpu(injected):
    native = injected
    items, expect = make_items(native, 40)
    good = [it for it, ok in zip(items, expect) if ok]
    bad = [it for it, ok in zip(items, expect) if not ok]
    before = native.sig_verify_stats()
    assert native.sig_batch_verify(good, use_gpu=True) is True
    assert native.sig_batch_verify(good + bad[:1], use_gpu=True) is False
    after = native.sig_verify_stats()
    assert after["gpu_failures"] - before["gpu_failures"] == 2
    assert after["cpu_sigs"] - before["cpu_sigs"] == 2 * len(good) + 1
    assert after["gpu_sigs"] == before["gpu_sigs"]
    assert not native.gpu_sig_path_disabled()
    # third consecutive failure switches the GPU path off; later batches go straight to the CPU
    assert native.sig_batch_verify(good, use_gpu=True) is True
    assert native.gpu_sig_path_disabled()
    n_fail = native.sig_verify_stats()["gpu_failures"]
    assert native.sig_batch_verify(good, use_gpu=True) is True
    assert native.sig_verify_stats()["gpu_failures"] == n_fail


def _solved_headers(native, count):
    out = []
    nonce = 0
    while len(out) < count:
        data = header_input(nonce, b"fallback")
        nonce += 1
        st = native.EquihashState(48, 5)
        st.update(data)
        sols, _ = native.eh_solve_cpu(48, 5, st)
        for s in sols[:1]:
            assert len(s) == 36
            out.append(data + bytes([len(s)]) + s)
    return out


def test_equihash_headers_fall_back_to_cpu(injected):
    native = injected
    hdrs = _solved_headers(native, 5)
    bad = bytearray(hdrs[0])
    bad[-1] ^= 0x01
    batch = hdrs + [bytes(bad)]
    expect = [True] * 5 + [False]
    assert native.check_equihash_headers(batch, "regtest", False) == expect
    assert native.check_equihash_headers(batch, "regtest", True) == expect


@pytest.mark.functional
def test_node_connects_blocks_when_gpu_fails(tmp_path):
    """A node that hits a GPU failure on every batch still syncs: node B has never seen the
    transactions (no signature-cache hits), so connecting A's block runs the batch path.
    Parity: reference validation.cpp:2121-2126 (post-fork script failures reject the block)."""
    from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess
    if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
        pytest.skip("bcpd not built")
    a = BcpdProcess(str(tmp_path / "a"), extra_args=["-gpu=0"])
    a.start()
    b = None
    try:
        # signature checks are deferred into the batch only post-fork (NULLFAIL), BCPHeight=3000
        a.rpc.generate(3001)
        addr = a.rpc.getnewaddress()
        for _ in range(6):
            a.rpc.sendtoaddress(addr, 1)
        tip = a.rpc.generate(1)[0]
        assert len(a.rpc.getblock(tip)["tx"]) == 7
        b = BcpdProcess(str(tmp_path / "b"), extra_args=["-gpufaultinjection", "-gpusigthreshold=1"])
        b.start()
        b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
        deadline = time.time() + 60
        while b.rpc.getbestblockhash() != tip:
            assert time.time() < deadline, "node B did not sync"
            time.sleep(0.2)
        sv = b.rpc.getgpuinfo()["sigverify"]
        assert sv["gpu_failures"] >= 1, (sv, b.rpc.getgpuinfo())
        assert sv["cpu_sigs"] >= 6
        assert sv["gpu_sigs"] == 0
    finally:
        if b is not None:
            b.stop()
        a.stop()
