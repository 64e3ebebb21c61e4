"""Contrib tooling: release hardening and symbol checks, option documentation, fixed seeds, rpcauth.

Parity:
* reference contrib/devtools/security-check.py with test-security-check.py: the four ELF checks
  pass on the release binaries and fail on deliberately unhardened builds;
* reference contrib/devtools/symbol-check.py and check-doc.py;
* reference contrib/seeds/{generate-seeds,makeseeds}.py;
* reference share/rpcauth/rpcauth.py: the line it prints authenticates against a real bcpd.
"""
import ipaddress
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = os.path.join(ROOT, "contrib", "devtools")
SEEDS = os.path.join(ROOT, "contrib", "seeds")
BIN = os.path.join(ROOT, "bin")

if not os.path.exists(os.path.join(BIN, "bcpd")):
    subprocess.check_call(["make", "-C", ROOT, "-j8", "tools"])


def run(*args, **kw):
    return subprocess.run([sys.executable, *args], capture_output=True, text=True, **kw)


RELEASE = [os.path.join(BIN, b) for b in ("bcpd", "bcp-cli", "bcp-tx", "bcp-seeder")] + \
          [os.path.join(ROOT, "lib", "libbcpconsensus.so")]


def test_security_check_passes_on_release_binaries():
    r = run(os.path.join(DEV, "security-check.py"), *[p for p in RELEASE if os.path.exists(p)])
    assert r.returncode == 0, r.stdout + r.stderr


def _cc(tmp_path, name, flags):
    src = tmp_path / "t.c"
    src.write_text("#include <stdio.h>\n#include <string.h>\n"
                   "int main(int c, char** v) { char b[64]; strcpy(b, v[0]); puts(b); return 0; }\n")
    out = tmp_path / name
    subprocess.check_call(["gcc", "-O1", "-o", str(out), str(src), *flags])
    return str(out)


def test_security_check_detects_each_missing_hardening(tmp_path):
    # reference test-security-check.py: build the same program without each protection
    chk = os.path.join(DEV, "security-check.py")
    good = _cc(tmp_path, "good", ["-fPIE", "-pie", "-fstack-protector-all", "-Wl,-z,relro,-z,now,-z,noexecstack"])
    assert run(chk, good).returncode == 0
    cases = {
        "PIE": ["-no-pie", "-fno-PIE", "-fstack-protector-all", "-Wl,-z,relro,-z,now"],
        "NX": ["-fPIE", "-pie", "-fstack-protector-all", "-Wl,-z,relro,-z,now,-z,execstack"],
        "RELRO": ["-fPIE", "-pie", "-fstack-protector-all", "-Wl,-z,norelro"],
        "Canary": ["-fPIE", "-pie", "-fno-stack-protector", "-Wl,-z,relro,-z,now"],
    }
    for want, flags in cases.items():
        exe = _cc(tmp_path, want.lower(), flags)
        r = run(chk, exe)
        assert r.returncode == 1, (want, r.stdout)
        assert want in r.stdout.split("failed", 1)[1].split(), (want, r.stdout)


def test_symbol_check():
    r = run(os.path.join(DEV, "symbol-check.py"), *[p for p in RELEASE if os.path.exists(p)])
    assert r.returncode == 0, r.stdout + r.stderr


def test_every_option_is_documented():
    r = run(os.path.join(DEV, "check-doc.py"), ROOT, "--reference")
    assert r.returncode == 0, r.stdout + r.stderr
    assert re.search(r"(\d+) options read, \d+ documented, 0 undocumented", r.stdout)
    # every option of the reference node is read or documented here (Qt-only switches aside)
    assert re.search(r"1\d\d reference options, 0 missing", r.stdout), r.stdout


def _parse_header(text):
    """(function name -> [(16 address bytes, port)]) from a generated chainparamsseeds.h."""
    out = {}
    for fn, body in re.findall(r"std::vector<SeedSpec6> (\w+)\(\) \{\s*return \{(.*?)\};", text, re.S):
        entries = []
        for addr, port in re.findall(r"\{\{([^}]*)\}, (\d+)\}", body):
            entries.append((bytes(int(x, 16) for x in addr.split(",")), int(port)))
        out[fn] = entries
    return out


def test_generate_seeds_encoding(tmp_path):
    (tmp_path / "nodes_main.txt").write_text(
        "# comment\n1.2.3.4\n5.6.7.8:9999\n[2001:db8::1]:8337\n2001:db8::2\n0x0100007f\n"
        "aaaaaaaaaaaaaaaa.onion:8333\n")
    (tmp_path / "nodes_test.txt").write_text("10.0.0.1\n")
    r = run(os.path.join(SEEDS, "generate-seeds.py"), str(tmp_path))
    assert r.returncode == 0, r.stderr
    seeds = _parse_header(r.stdout)
    main = seeds["FixedSeedsMain"]
    v4 = lambda s: bytes(10) + b"\xff\xff" + ipaddress.IPv4Address(s).packed
    assert main[0] == (v4("1.2.3.4"), 8337)
    assert main[1] == (v4("5.6.7.8"), 9999)
    assert main[2] == (ipaddress.IPv6Address("2001:db8::1").packed, 8337)
    assert main[3] == (ipaddress.IPv6Address("2001:db8::2").packed, 8337)
    assert main[4] == (v4("127.0.0.1"), 8337)
    assert main[5][0][:6] == bytes([0xFD, 0x87, 0xD8, 0x7E, 0xEB, 0x43]) and main[5][1] == 8333
    assert seeds["FixedSeedsTest"] == [(v4("10.0.0.1"), 18337)]


def test_in_tree_seeds_header_is_current():
    r = run(os.path.join(SEEDS, "generate-seeds.py"), SEEDS)
    assert r.returncode == 0
    with open(os.path.join(ROOT, "csrc", "consensus", "chainparamsseeds.h")) as f:
        assert f.read() == r.stdout, "regenerate csrc/consensus/chainparamsseeds.h (contrib/seeds/README.md)"


def test_makeseeds_filters_and_diversifies():
    hdr = "# address                                        good  lastSuccess    %(2h)  blocks      svcs  version\n"
    rows = [
        ("1.2.3.4:8337", 1, 99.0, 600000, 0x25, 70016, "/Bitcoin Cash Plus:0.17.0/"),
        ("1.2.9.9:8337", 1, 98.0, 600000, 0x25, 70016, "/Bitcoin Cash Plus:0.17.0/"),
        ("1.2.7.7:8337", 1, 97.0, 600000, 0x25, 70016, "/Bitcoin Cash Plus:0.17.0/"),  # third in 1.2/16
        ("5.5.5.5:8337", 0, 99.0, 600000, 0x25, 70016, "/Bitcoin Cash Plus:0.17.0/"),  # not good
        ("6.6.6.6:8337", 1, 20.0, 600000, 0x25, 70016, "/Bitcoin Cash Plus:0.17.0/"),  # low uptime
        ("7.7.7.7:8337", 1, 99.0, 600000, 0x24, 70016, "/Bitcoin Cash Plus:0.17.0/"),  # no NODE_NETWORK
        ("8.8.8.8:8337", 1, 99.0, 100, 0x25, 70016, "/Bitcoin Cash Plus:0.17.0/"),  # too low
        ("9.9.9.9:8337", 1, 99.0, 600000, 0x25, 70015, "/Bitcoin Cash Plus:0.17.0/"),  # legacy protocol
        ("10.1.1.1:8337", 1, 99.0, 600000, 0x25, 70016, "/Satoshi:0.16.0/"),  # other agent
        ("[2001:db8::5]:8337", 1, 95.0, 600000, 0x25, 70016, "/Bitcoin Cash Plus:0.17.0/"),
    ]
    dump = hdr + "".join(f'{a:<47s}  {g:4d}  {1600000000:11d}  {u:6.2f}%  {b:6d}  {s:08x}  {v:5d} "{ag}"\n'
                         for a, g, u, b, s, v, ag in rows)
    r = run(os.path.join(SEEDS, "makeseeds.py"), "--min-blocks", "500000", input=dump)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["1.2.3.4:8337", "1.2.9.9:8337", "[2001:db8::5]:8337"]


def test_rpcauth_line_authenticates(tmp_path):
    sys.path.insert(0, ROOT)
    from bitcoincashplus_amd.node.process import BcpdProcess, RPCProxy
    r = run(os.path.join(ROOT, "share", "rpcauth", "rpcauth.py"), "alice", "s3cret-pass")
    line = next(l for l in r.stdout.splitlines() if l.startswith("rpcauth="))
    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-" + line])
    n.start()
    try:
        assert RPCProxy(n.rpcport, "alice", "s3cret-pass").getblockcount() == 0
        with pytest.raises(Exception):
            RPCProxy(n.rpcport, "alice", "wrong").getblockcount()
    finally:
        n.stop()
