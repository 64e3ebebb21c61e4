"""Outbound SOCKS5 proxying and -onlynet (reference qa/rpc-tests/proxy_test.py): a Python
SOCKS5 server relays node A's connection to node B; it must see the destination as a
domain-name CONNECT (no local resolution), random credentials per connection under
-proxyrandomize, and getnetworkinfo must report the proxy per network. -onlynet=onion keeps
the node from dialing an IPv4 peer directly."""
import os
import socket
import struct
import threading
import time

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess

pytestmark = pytest.mark.functional

if not os.path.exists(os.path.join(BIN_DIR, "bcpd")):
    import subprocess
    subprocess.check_call(["make", "-C", os.path.dirname(BIN_DIR), "-j8", "tools"])


class Socks5Relay:
    """Minimal SOCKS5 server: records each CONNECT, then pipes bytes to the real target."""

    def __init__(self):
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(8)
        self.port = self.srv.getsockname()[1]
        self.requests = []  # (atyp, host, port, username)
        self.stop = False
        threading.Thread(target=self._accept, daemon=True).start()

    def _recv(self, c, n):
        b = b""
        while len(b) < n:
            x = c.recv(n - len(b))
            if not x:
                raise ConnectionError
            b += x
        return b

    def _accept(self):
        while not self.stop:
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c):
        try:
            ver, nm = self._recv(c, 2)
            methods = self._recv(c, nm)
            user = None
            if 2 in methods:
                c.sendall(b"\x05\x02")
                _, ul = self._recv(c, 2)
                user = self._recv(c, ul).decode()
                (pl,) = self._recv(c, 1)
                self._recv(c, pl)
                c.sendall(b"\x01\x00")
            else:
                c.sendall(b"\x05\x00")
            ver, cmd, _, atyp = self._recv(c, 4)
            if atyp == 3:
                (ln,) = self._recv(c, 1)
                host = self._recv(c, ln).decode()
            elif atyp == 1:
                host = socket.inet_ntoa(self._recv(c, 4))
            else:
                host = socket.inet_ntop(socket.AF_INET6, self._recv(c, 16))
            (port,) = struct.unpack(">H", self._recv(c, 2))
            self.requests.append((atyp, host, port, user))
            up = socket.create_connection(("127.0.0.1", port), timeout=10)
            c.sendall(b"\x05\x00\x00\x01" + socket.inet_aton("127.0.0.1") + struct.pack(">H", port))
            for a, b in ((c, up), (up, c)):
                threading.Thread(target=self._pipe, args=(a, b), daemon=True).start()
        except Exception:
            c.close()

    @staticmethod
    def _pipe(a, b):
        try:
            while True:
                d = a.recv(65536)
                if not d:
                    break
                b.sendall(d)
        except OSError:
            pass
        finally:
            for s in (a, b):
                try:
                    s.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass

    def close(self):
        self.stop = True
        self.srv.close()


def wait_until(pred, timeout=60):
    end = time.time() + timeout
    while time.time() < end:
        if pred():
            return
        time.sleep(0.1)
    raise AssertionError("timed out")


def test_connect_through_socks5_proxy(tmp_path):
    relay = Socks5Relay()
    b = BcpdProcess(str(tmp_path / "b"), extra_args=["-gpu=0"])
    a = BcpdProcess(str(tmp_path / "a"), extra_args=["-gpu=0", f"-proxy=127.0.0.1:{relay.port}", "-listen=0"])
    b.start()
    a.start()
    try:
        nets = {n["name"]: n for n in a.rpc.getnetworkinfo()["networks"]}
        assert nets["ipv4"]["proxy"] == f"127.0.0.1:{relay.port}"
        assert nets["ipv4"]["proxy_randomize_credentials"] is True
        b.rpc.generate(5)
        a.rpc.addnode(f"localhost:{b.p2p_port}", "onetry")
        wait_until(lambda: a.rpc.getblockcount() == 5)
        # the name went to the proxy unresolved, with per-connection random credentials
        atyp, host, port, user = relay.requests[0]
        assert (atyp, host, port) == (3, "localhost", b.p2p_port)
        assert user and len(user) == 8
    finally:
        a.stop()
        b.stop()
        relay.close()


def test_onlynet_and_onion_reachability(tmp_path):
    """-onlynet=onion marks IPv4/IPv6 limited (automatic outbound skips them; like the
    reference, local/unroutable addresses are not subject to it); without -proxy/-onion no
    onion peer is reachable; an unknown network name is a startup error."""
    a = BcpdProcess(str(tmp_path / "a"), extra_args=["-gpu=0", "-onlynet=onion", "-onion=127.0.0.1:9", "-listen=0"])
    a.start()
    try:
        nets = {n["name"]: n for n in a.rpc.getnetworkinfo()["networks"]}
        assert nets["ipv4"]["limited"] and not nets["ipv4"]["reachable"]
        assert nets["ipv6"]["limited"]
        assert nets["onion"]["reachable"] and nets["onion"]["proxy"] == "127.0.0.1:9"
    finally:
        a.stop()
    c = BcpdProcess(str(tmp_path / "c"), extra_args=["-gpu=0", "-listen=0"])
    c.start()
    try:
        nets = {n["name"]: n for n in c.rpc.getnetworkinfo()["networks"]}
        assert nets["ipv4"]["reachable"] and not nets["onion"]["reachable"]
    finally:
        c.stop()
    d = BcpdProcess(str(tmp_path / "d"), extra_args=["-gpu=0", "-onlynet=carrierpigeon"])
    with pytest.raises(RuntimeError):
        d.start()
