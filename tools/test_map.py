#!/usr/bin/env python3
"""Writes docs/TEST_MAP.md: every reference functional script and unit suite, and the test
files here that port it (found by the reference file name they cite), or why none does.

    python3 tools/test_map.py [/root/reference]
"""
import glob
import os
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# reference files with no port, and why
NOT_PORTED = {
    "create_cache.py": "framework helper (builds the 200-block cache); tests mine their own chains",
    "test_runner.py": "framework runner; pytest runs the suite (`pytest tests -m 'not gpu'`)",
    "reverselock_tests.cpp": "no reverse_lock helper here",
    "raii_event_tests.cpp": "libevent RAII wrappers; the HTTP server here does not use libevent",
    "scriptflags.cpp": "helper of script_tests (flag-name parsing), used by tests/test_script.py",
    "sigutil.cpp": "helper of sighash tests",
    "testutil.cpp": "helper (temp paths)",
    "wallet_test_fixture.cpp": "fixture; csrc/test/unittest.h has the equivalents",
    "test_bitcoin.cpp": "fixture; csrc/test/test_main.cpp",
    "test_bitcoin_fuzzy.cpp": "fuzz harness; bin/bcp-fuzz + tests/test_fuzz.py",
    "test_bitcoin_main.cpp": "runner; csrc/test/test_main.cpp",
    "test_random.h": "helper",
}


def ours():
    files = glob.glob(os.path.join(ROOT, "tests", "*.py")) + glob.glob(os.path.join(ROOT, "csrc", "test", "*.cpp"))
    return {os.path.relpath(p, ROOT): open(p, errors="replace").read() for p in sorted(files)}


def cites(name, texts):
    stem = os.path.splitext(name)[0]
    keys = {name}
    if name.endswith(".cpp"):
        keys.add(stem)  # "multisig_tests" as a suite name
    return [p for p, t in texts.items() if any(k in t for k in keys)]


def table(title, names, texts):
    lines = [f"## {title}", "", "| reference | ported in |", "|---|---|"]
    done = 0
    for n in names:
        hits = cites(n, texts)
        if hits:
            done += 1
            cell = ", ".join(f"`{h}`" for h in hits[:4]) + (f" (+{len(hits) - 4})" if len(hits) > 4 else "")
        else:
            cell = "not ported: " + NOT_PORTED.get(n, "**missing**")
        lines.append(f"| `{n}` | {cell} |")
    lines.append("")
    lines.append(f"{done} of {len(names)} cited by a test here.")
    lines.append("")
    return lines


# Per-case checklist for the largest reference scripts: (case, reference lines, our test as
# "file::function" or None, note). Every named test function must exist (checked below).
CASES = {
    "p2p-compactblocks.py": [
        ("test_sendcmpct (negotiation, announcements)", "171-276", "tests/test_p2p_compactblocks.py::test_sendcmpct_and_announcements", ""),
        ("test_invalid_cmpctblock_message", "278-290", "tests/test_p2p_compactblocks_cases.py::test_invalid_cmpctblock_message", ""),
        ("test_compactblock_construction (short ids)", "294-398", "tests/test_p2p_compactblocks.py::test_sendcmpct_and_announcements", "SipHash short ids checked independently"),
        ("test_compactblock_requests (node reconstructs)", "400-469", "tests/test_p2p_compactblocks.py::test_node_reconstructs_compact_block", ""),
        ("test_getblocktxn_requests", "471-564", "tests/test_p2p_compactblocks.py::test_node_reconstructs_compact_block", "getblocktxn for exactly the missing indexes"),
        ("test_incorrect_blocktxn_response", "566-627", "tests/test_p2p_compactblocks_cases.py::test_incorrect_blocktxn_response", "plus the wrong-count misbehaviour"),
        ("test_getblocktxn_handler (depth 10)", "629-682", "tests/test_p2p_compactblocks_cases.py::test_getblocktxn_handler", ""),
        ("test_compactblocks_not_at_tip (depth 5)", "684-741", "tests/test_p2p_compactblocks_cases.py::test_compactblocks_not_at_tip", ""),
        ("test_end_to_end_block_relay", "744-762", "tests/test_p2p_compactblocks.py::test_sendcmpct_and_announcements", "a mined block reaches a high-bandwidth peer as cmpctblock"),
        ("test_invalid_tx_in_compactblock", "764-784", "tests/test_p2p_compactblocks_cases.py::test_invalid_tx_in_compactblock", ""),
        ("test_compactblock_reconstruction_multiple_peers", "796-850", "tests/test_p2p_compactblocks_cases.py::test_compactblock_reconstruction_multiple_peers", "BCH analogue of the witness corruption"),
        ("segwit (version 2) variants", "-", None, "n/a: no segregated witness on this chain"),
    ],
    "sendheaders.py": [
        ("Part 1: no headers announcements before sendheaders", "300-334", "tests/test_p2p_sendheaders.py::test_sendheaders_parts_1_to_5", ""),
        ("Part 2: headers announcements after sendheaders", "336-402", "tests/test_p2p_sendheaders.py::test_sendheaders_parts_1_to_5", ""),
        ("Part 3: large reorg -> inv; resume after getheaders / inv", "405-476", "tests/test_p2p_sendheaders.py::test_sendheaders_parts_1_to_5", ""),
        ("Part 4: direct fetch", "478-566", "tests/test_p2p_sendheaders.py::test_sendheaders_parts_1_to_5", ""),
        ("Part 5: unconnecting headers, disconnect after 5 x 10", "571-643", "tests/test_p2p_sendheaders.py::test_sendheaders_parts_1_to_5", ""),
    ],
    "fundrawtransaction.py": [
        (c, "", "tests/test_functional_fundraw.py::test_fundrawtransaction", "") for c in (
            "simple test / two coins / two outputs", "VIN greater than required", "no change output",
            "invalid option", "invalid change address", "provided change address / changePosition",
            "VIN smaller than required", "two VINs / two VINs and two vOUTs", "invalid vin",
            "fee comparisons (P2PKH, multiple outputs, 2of2, 4of5)", "spend a 2of2 multisig",
            "locked wallet", "~19 inputs: fee / sign and send", "OP_RETURN and no vin", "watch-only",
            "entirety of watched funds", "feeRate", "reserveChangeKey", "subtractFeeFromOutputs")
    ],
    "bip68-112-113-p2p.py": [
        ("deployment: DEFINED/STARTED/LOCKED_IN (TestInstances 1-5)", "231-321", "tests/test_p2p_bip68_112_113.py::test_bip68_112_113", "run 20 periods later, past the fork"),
        ("before activation: all pass (6-7)", "369-417", "tests/test_p2p_bip68_112_113.py::test_bip68_112_113", ""),
        ("BIP113 (9-12)", "421-441", "tests/test_p2p_bip68_112_113.py::test_bip68_112_113", ""),
        ("BIP68 version 1 / 2, height and time locks (14-31)", "447-498", "tests/test_p2p_bip68_112_113.py::test_bip68_112_113", ""),
        ("BIP112 version 1 (32-81)", "500-530", "tests/test_p2p_bip68_112_113.py::test_bip68_112_113", ""),
        ("BIP112 version 2 (82-125)", "532-607", "tests/test_p2p_bip68_112_113.py::test_bip68_112_113", ""),
    ],
}


def fullblock_cases(texts):
    """p2p-fullblocktest.py: one case per numbered block of the reference; ported when our
    fullblock tests build a block of that number."""
    import re
    ref = open(os.path.join(REF, "test", "functional", "p2p-fullblocktest.py")).read()
    ours = texts.get("tests/test_p2p_fullblock.py", "")
    label = re.compile(r"""block\((\d+|"[0-9a-z]+")""")
    theirs = sorted({m.group(1).strip('"') for m in label.finditer(ref)}, key=lambda x: (len(x), x))
    mine = {m.group(1).strip('"') for m in label.finditer(ours)}
    # blocks our port builds by another route than block(N) (text that shows where, and a note)
    aliases = {
        "56": ("b56 = CBlock(b57", "b57's header with a duplicated transaction (CVE-2012-2459)"),
        "b56p2": ("b56p2 = CBlock(b57p2", "non-adjacent duplicates, same merkle root"),
        "64": ("bloated", "the canonical re-serialisation of b64a"),
        "alt": ("a longer reorg back and forth", "150-block chains where the reference uses 1088"),
    }
    rows = []
    for b in theirs:
        if b in mine:
            rows.append((f"b{b}", "", "tests/test_p2p_fullblock.py::test_fullblock_prefork", ""))
        elif b in aliases and aliases[b][0] in ours:
            rows.append((f"b{b}", "", "tests/test_p2p_fullblock.py::test_fullblock_prefork", aliases[b][1]))
        else:
            rows.append((f"b{b}", "", None, "not built by our port"))
    return rows


def case_tables(texts):
    lines = ["## Case checklist for the largest scripts", "",
             "One row per case of the reference script; the named test function asserts that case's",
             "outcome (messages, reject or misbehaviour, announcement type). `tools/test_map.py` checks",
             "that every named function exists.", ""]
    allcases = dict(CASES)
    allcases["p2p-fullblocktest.py"] = fullblock_cases(texts)
    for script, rows in allcases.items():
        done = sum(1 for r in rows if r[2])
        lines += [f"### `{script}` ({done} of {len(rows)} cases ported)", "", "| case | reference lines | test here | note |",
                  "|---|---|---|---|"]
        for case, where, test, note in rows:
            if test:
                f, _, fn = test.partition("::")
                if f"def {fn}(" not in texts.get(f, ""):
                    raise SystemExit(f"test_map: {test} named for {script} does not exist")
            lines.append(f"| {case} | {where} | {'`' + test + '`' if test else 'not ported'} | {note} |")
        lines.append("")
    return lines


def main():
    texts = ours()
    func = sorted(os.path.basename(p) for p in glob.glob(os.path.join(REF, "test", "functional", "*.py")))
    unit = sorted(os.path.basename(p) for p in glob.glob(os.path.join(REF, "src", "test", "*.cpp")))
    wunit = sorted(os.path.basename(p) for p in glob.glob(os.path.join(REF, "src", "wallet", "test", "*.cpp")))
    out = ["# Reference tests and their ports", "",
           "Generated by `tools/test_map.py` from the file names each test here cites in its docstring or",
           "header comment (\"Parity: reference ...\"). A reference file is listed as ported when at least one",
           "test names it; the named tests assert that file's outputs and reject reasons. The five largest",
           "scripts also get a per-case checklist at the end.", ""]
    out += table("Functional scripts (`test/functional/`)", func, texts)
    out += table("Unit suites (`src/test/`)", unit, texts)
    out += table("Wallet unit suites (`src/wallet/test/`)", wunit, texts)
    out += case_tables(texts)
    with open(os.path.join(ROOT, "docs", "TEST_MAP.md"), "w") as f:
        f.write("\n".join(out))
    print("\n".join(l for l in out if "**missing**" in l) or "nothing missing")


if __name__ == "__main__":
    main()
