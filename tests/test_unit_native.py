"""Runs the native unit suites of bin/test_bcp (csrc/test/*.cpp), one pytest case per suite.

Parity: reference src/test/ Boost suites run by test_bitcoin (each suite's cases cite the
reference file they port)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin", "test_bcp")


def _suites():
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-C", ROOT, "-j8", "unittest"])
    out = subprocess.run([BIN, "--list"], capture_output=True, text=True, check=True).stdout
    return [l.split()[0] for l in out.splitlines() if l.strip()]


SUITES = _suites()


def test_suite_inventory():
    # the suites ported from reference src/test/ (each must exist and hold cases)
    for s in [
        "script_antireplay_tests", "sigopcount_tests", "bloom_tests", "pmt_tests", "blockencodings_tests",
        "coins_tests", "versionbits_tests", "mempool_tests", "kvstore_tests", "sigbatch_tests", "miner_tests",
        "policyestimator_tests", "txvalidationcache_tests", "addrman_tests", "crypto_tests", "dos_tests", "checkqueue_tests",
        "getarg_tests", "util_tests", "timedata_tests", "netbase_tests", "serialize_tests", "streams_tests",
        "compress_tests", "rpc_tests", "skiplist_tests", "wallet_tests", "walletdb_tests", "connectblock_tests", "blockdecode_tests", "net_tests", "blockcheck_tests",
        "validation_tests", "modinv_tests", "derlax_tests", "scriptnum_tests", "script_sighashtype_tests",
        "multisig_tests", "shardplan_tests",
    ]:
        assert s in SUITES, s


@pytest.mark.parametrize("suite", SUITES)
def test_native_suite(suite, tmp_path):
    p = subprocess.run([BIN, f"--suite={suite}"], capture_output=True, text=True, cwd=str(tmp_path), timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "0 failed" in p.stdout
