"""bcp-seeder (reference src/seeder): crawls a live regtest bcpd over P2P, marks it good,
and serves it in A-record answers for the seed zone; NS/SOA answers and REFUSED for
out-of-zone names."""
import os
import socket
import struct
import subprocess
import time

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess, free_port

pytestmark = pytest.mark.functional


def dns_query(port, name, qtype):
    q = struct.pack(">HHHHHH", 0x1234, 0x0100, 1, 0, 0, 0)
    for part in name.split("."):
        q += bytes([len(part)]) + part.encode()
    q += b"\x00" + struct.pack(">HH", qtype, 1)
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.settimeout(3)
    s.sendto(q, ("127.0.0.1", port))
    r, _ = s.recvfrom(1500)
    rid, flags, qd, an, ns, ar = struct.unpack(">HHHHHH", r[:12])
    assert rid == 0x1234
    off = 12 + len(q) - 12  # skip the echoed question
    answers = []
    for _ in range(an):
        off += 2  # name pointer
        typ, cls, ttl, rdlen = struct.unpack(">HHIH", r[off:off + 10])
        off += 10
        answers.append((typ, r[off:off + rdlen]))
        off += rdlen
    return flags & 0xF, answers


def test_seeder_crawls_and_answers(tmp_path):
    node = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0"])
    node.start()
    dns_port = free_port()
    dump = str(tmp_path / "seed.dump")
    p = subprocess.Popen([os.path.join(BIN_DIR, "bcp-seeder"), "-regtest", "-host=seed.bcp.test", "-ns=ns.bcp.test",
                          f"-port={dns_port}", "-threads=2", f"-seed=127.0.0.1:{node.p2p_port}", "-allowlocal",
                          f"-dumpfile={dump}", "-dumpinterval=1"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        deadline = time.time() + 30
        answers = []
        while time.time() < deadline:
            try:
                rc, answers = dns_query(dns_port, "seed.bcp.test", 1)
            except OSError:  # seeder not bound yet
                time.sleep(0.3)
                continue
            if answers:
                break
            time.sleep(0.3)
        assert rc == 0 and answers and answers[0] == (1, socket.inet_aton("127.0.0.1"))
        rc, ns = dns_query(dns_port, "seed.bcp.test", 2)
        assert ns and ns[0][0] == 2
        rc, soa = dns_query(dns_port, "seed.bcp.test", 6)
        assert soa and soa[0][0] == 6
        rc, _ = dns_query(dns_port, "other.example", 1)
        assert rc == 5  # REFUSED
        text = ""
        deadline = time.time() + 20  # the dumper writes every -dumpinterval seconds
        while time.time() < deadline:
            if os.path.exists(dump):
                text = open(dump).read()
                if f"127.0.0.1:{node.p2p_port}" in text:
                    break
            time.sleep(0.3)
        assert f"127.0.0.1:{node.p2p_port}" in text and "/Bitcoin Cash Plus:" in text
    finally:
        p.terminate()
        p.wait(20)
        node.stop()
