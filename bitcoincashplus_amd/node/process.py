"""Out-of-process node driver for functional tests (reference qa/rpc-tests/
test_framework/{test_node,util,authproxy}.py: start bitcoind with -datadir/-rpcport,
wait for RPC, call over HTTP JSON-RPC with Basic auth, stop via the `stop` RPC).

    with BcpdProcess(tmpdir, extra_args=["-gpu=0"]) as n:
        n.rpc.generate(5)
"""
from __future__ import annotations

import base64
import http.client
import json
import os
import socket
import subprocess
import time

from .embedded import RPCError

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN_DIR = os.path.join(ROOT, "bin")


def free_port() -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _json_default(o):
    """Decimal amounts travel as JSON numbers (reference authproxy EncodeDecimal)."""
    import decimal
    if isinstance(o, decimal.Decimal):
        return float(o)
    raise TypeError(f"{type(o).__name__} is not JSON serializable")


class RPCProxy:
    """Minimal JSON-RPC-over-HTTP client (reference authproxy.AuthServiceProxy)."""

    def __init__(self, port, user, password, path="/", timeout=120):
        self.port = port
        self.path = path
        self.auth = "Basic " + base64.b64encode(f"{user}:{password}".encode()).decode()
        self.timeout = timeout
        self._id = 0

    def _post(self, body: str):
        conn = http.client.HTTPConnection("127.0.0.1", self.port, timeout=self.timeout)
        try:
            conn.request("POST", self.path, body, {"Authorization": self.auth, "Content-Type": "application/json"})
            resp = conn.getresponse()
            return resp.status, resp.read().decode()
        finally:
            conn.close()

    def call(self, method, *params, **named):
        self._id += 1
        req = {"version": "1.1", "method": method, "params": named if named else list(params), "id": self._id}
        status, text = self._post(json.dumps(req, default=_json_default))
        if status == 401:
            raise RPCError(-1, "authorization failed")
        reply = json.loads(text)
        if reply.get("error"):
            raise RPCError(reply["error"]["code"], reply["error"]["message"])
        return reply["result"]

    def batch(self, calls):
        body = json.dumps([{"method": m, "params": list(p), "id": i} for i, (m, p) in enumerate(calls)])
        status, text = self._post(body)
        return json.loads(text)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return lambda *p, **kw: self.call(name, *p, **kw)


class BcpdProcess:
    def __init__(self, datadir, chain="regtest", extra_args=(), rpcuser="rt", rpcpassword="rtpass", port=None,
                 p2p_port=None, binary=None):
        self.datadir = datadir
        self.chain = chain
        self.rpcport = port or free_port()
        self.p2p_port = p2p_port or free_port()
        self.user, self.password = rpcuser, rpcpassword
        # BCP_BCPD: run another build of the node (e.g. bin/tsan/bcpd, tools/sanitize.sh)
        self.binary = binary or os.environ.get("BCP_BCPD") or os.path.join(BIN_DIR, "bcpd")
        self.extra_args = list(extra_args)
        self.proc = None
        self.rpc = RPCProxy(self.rpcport, rpcuser, rpcpassword)
        os.makedirs(datadir, exist_ok=True)

    def args(self):
        chainflag = {"regtest": ["-regtest"], "test": ["-testnet"], "main": []}[self.chain]
        return [self.binary, f"-datadir={self.datadir}", *chainflag, f"-rpcport={self.rpcport}",
                f"-port={self.p2p_port}", f"-rpcuser={self.user}", f"-rpcpassword={self.password}",
                "-listenonion=0", "-discover=0", "-dnsseed=0", "-debuglockorder=1", *self.extra_args]

    def start(self, wait=True, timeout=60):
        log = open(os.path.join(self.datadir, "stdout.log"), "ab")
        self.proc = subprocess.Popen(self.args(), stdout=log, stderr=subprocess.STDOUT)
        if wait:
            self.wait_for_rpc(timeout)
        return self

    def wait_for_rpc(self, timeout=60):
        deadline = time.time() + timeout
        last = None
        while time.time() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError(f"bcpd exited with {self.proc.returncode}: {self.tail_log()}")
            try:
                self.rpc.getblockcount()
                return
            except RPCError as e:
                last = e
                if e.code != -28:  # RPC_IN_WARMUP
                    raise
            except (ConnectionError, OSError) as e:
                last = e
            time.sleep(0.1)
        raise TimeoutError(f"bcpd RPC not up after {timeout}s: {last}")

    def tail_log(self, n=4000):
        path = os.path.join(self.datadir, "stdout.log")
        try:
            with open(path, "rb") as f:
                return f.read()[-n:].decode(errors="replace")
        except OSError:
            return ""

    def stop(self, timeout=60):
        if not self.proc or self.proc.poll() is not None:
            return
        try:
            self.rpc.stop()
        except Exception:
            self.proc.terminate()
        try:
            self.proc.wait(timeout)
        except subprocess.TimeoutExpired:
            self.proc.kill()
            self.proc.wait()

    def cli(self, *args, check=True):
        cmd = [os.path.join(BIN_DIR, "bcp-cli"), f"-datadir={self.datadir}",
               {"regtest": "-regtest", "test": "-testnet", "main": ""}[self.chain] or "-rpcwait",
               f"-rpcport={self.rpcport}", f"-rpcuser={self.user}", f"-rpcpassword={self.password}", *args]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        if check and r.returncode != 0:
            raise RuntimeError(f"bcp-cli {args} -> {r.returncode}: {r.stderr}")
        return r

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
