"""Tor control-port integration (reference src/torcontrol.cpp behaviour) against a fake
Tor controller: PROTOCOLINFO, SAFECOOKIE challenge/response (HMAC-SHA256 with the fixed
Tor keys), ADD_ONION with key persistence, and the onion address advertised as a local
address in getnetworkinfo."""
import hashlib
import hmac
import os
import socket
import threading
import time

import pytest

from bitcoincashplus_amd.node.process import BcpdProcess

pytestmark = pytest.mark.functional

SERVER_KEY = b"Tor safe cookie authentication server-to-controller hash"
CLIENT_KEY = b"Tor safe cookie authentication controller-to-server hash"


class FakeTor(threading.Thread):
    def __init__(self, cookie_path):
        super().__init__(daemon=True)
        self.cookie = os.urandom(32)
        open(cookie_path, "wb").write(self.cookie)
        self.cookie_path = cookie_path
        self.srv = socket.socket()
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(1)
        self.port = self.srv.getsockname()[1]
        self.commands = []
        self.authed = False

    def run(self):
        conn, _ = self.srv.accept()
        f = conn.makefile("rwb")
        snonce = os.urandom(32)
        cnonce = None
        while True:
            line = f.readline()
            if not line:
                return
            cmd = line.decode().strip()
            self.commands.append(cmd)
            if cmd.startswith("PROTOCOLINFO"):
                f.write(b'250-PROTOCOLINFO 1\r\n250-AUTH METHODS=COOKIE,SAFECOOKIE COOKIEFILE="%s"\r\n'
                        b'250-VERSION Tor="0.3.5.8"\r\n250 OK\r\n' % self.cookie_path.encode())
            elif cmd.startswith("AUTHCHALLENGE SAFECOOKIE"):
                cnonce = bytes.fromhex(cmd.split()[2])
                sh = hmac.new(SERVER_KEY, self.cookie + cnonce + snonce, hashlib.sha256).hexdigest()
                f.write(("250 AUTHCHALLENGE SERVERHASH=%s SERVERNONCE=%s\r\n" % (sh, snonce.hex())).encode())
            elif cmd.startswith("AUTHENTICATE"):
                want = hmac.new(CLIENT_KEY, self.cookie + cnonce + snonce, hashlib.sha256).hexdigest()
                self.authed = cmd.split()[1].lower() == want
                f.write(b"250 OK\r\n" if self.authed else b"515 Authentication failed\r\n")
            elif cmd.startswith("ADD_ONION"):
                f.write(b"250-ServiceID=abcdefghijklmnop\r\n250-PrivateKey=RSA1024:SECRETKEY\r\n250 OK\r\n")
            else:
                f.write(b"510 Unrecognized command\r\n")
            f.flush()


def test_onion_service_registration(tmp_path):
    tor = FakeTor(str(tmp_path / "control_auth_cookie"))
    tor.start()
    n = BcpdProcess(str(tmp_path / "t"), extra_args=["-gpu=0", "-listenonion=1", f"-torcontrol=127.0.0.1:{tor.port}"])
    n.start()
    try:
        deadline = time.time() + 20
        locals_ = []
        while time.time() < deadline:
            locals_ = n.rpc.getnetworkinfo()["localaddresses"]
            if locals_:
                break
            time.sleep(0.2)
        assert tor.authed
        assert any(c.startswith("ADD_ONION NEW:RSA1024 Port=%d,127.0.0.1:%d" % (n.p2p_port, n.p2p_port))
                   for c in tor.commands)
        assert locals_ and locals_[0]["address"] == "abcdefghijklmnop.onion" and locals_[0]["port"] == n.p2p_port
        assert open(os.path.join(n.datadir, "regtest", "onion_private_key")).read().strip() == "RSA1024:SECRETKEY"
    finally:
        n.stop()
