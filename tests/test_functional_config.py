"""Node options that round 4 brought to the reference's set (reference src/init.cpp,
src/wallet/wallet.cpp, src/httpserver.cpp, src/rpc/protocol.cpp, src/miner.cpp), end to end on a
regtest bcpd:

* -rpccookiefile (absolute and datadir-relative; bcp-cli finds it too), -rpcworkqueue
  ("Work queue depth exceeded" once -rpcthreads + -rpcworkqueue requests are in flight);
* -mocktime (the node's clock, e.g. the first block's time), -stopafterblockimport with
  -loadblock (the node imports, then shuts down by itself);
* obsolete options: -socks / -tor / -rpcssl stop startup with the reference's messages,
  -benchmark / -debugnet / -blockminsize / -whitelistalwaysrelay only warn;
* -sysperms (umask 077 otherwise; refused with a wallet);
* -upgradewallet / wallet versions (HD 130000, non-HD 60000, "Cannot downgrade wallet"),
  -sendfreetransactions needs -limitfreerelay, -walletrejectlongchains refuses a send that
  would exceed the mempool's chain limits;
* -printpriority logs each mined transaction's priority and fee, -help-debug lists the
  debugging options, -dns=0 refuses to resolve -addnode names.
contrib/devtools/check-doc.py --reference (tests/test_contrib_tools.py) checks the option
list itself against the reference's.
"""
import os
import stat
import subprocess
import threading
import time

import pytest

from bitcoincashplus_amd.node.process import BIN_DIR, BcpdProcess, RPCError, RPCProxy, free_port

pytestmark = pytest.mark.functional


def node(tmp_path, name, *args):
    n = BcpdProcess(str(tmp_path / name), extra_args=["-gpu=0", *args])
    n.start()
    return n


def run_to_exit(tmp_path, name, *args, timeout=60):
    d = tmp_path / name
    d.mkdir(exist_ok=True)
    n = BcpdProcess(str(d), extra_args=["-gpu=0", *args])
    r = subprocess.run(n.args(), capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr, n


def wait_until(pred, timeout=30):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(0.05)
    return False


def debug_log(n):
    with open(os.path.join(n.datadir, "regtest", "debug.log"), errors="replace") as f:
        return f.read()


def test_rpccookiefile(tmp_path):
    for cookie in ("mycookie", str(tmp_path / "abs.cookie")):
        d = tmp_path / ("d" + str(abs(hash(cookie)) % 1000))
        d.mkdir()
        port = free_port()
        args = [os.path.join(BIN_DIR, "bcpd"), f"-datadir={d}", "-regtest", f"-rpcport={port}", f"-port={free_port()}",
                "-gpu=0", "-listenonion=0", "-dnsseed=0", "-discover=0", f"-rpccookiefile={cookie}"]
        p = subprocess.Popen(args, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        try:
            path = cookie if os.path.isabs(cookie) else str(d / "regtest" / cookie)
            assert wait_until(lambda: os.path.exists(path))
            assert not os.path.exists(d / "regtest" / ".cookie")
            user, pw = open(path).read().strip().split(":", 1)
            assert user == "__cookie__"
            rpc = RPCProxy(port, user, pw)
            assert wait_until(lambda: _ok(rpc.getblockcount))
            r = subprocess.run([os.path.join(BIN_DIR, "bcp-cli"), f"-datadir={d}", "-regtest", f"-rpcport={port}",
                                f"-rpccookiefile={cookie}", "getblockcount"], capture_output=True, text=True, timeout=60)
            assert r.returncode == 0 and r.stdout.strip() == "0", r.stderr
            rpc.stop()
            p.wait(60)
            assert not os.path.exists(path)  # removed at shutdown
        finally:
            if p.poll() is None:
                p.kill()
                p.wait()


def _ok(fn):
    try:
        fn()
        return True
    except Exception:
        return False


def test_rpcworkqueue(tmp_path):
    n = node(tmp_path, "n", "-rpcthreads=1", "-rpcworkqueue=1")
    try:
        n.rpc.generate(1)
        results = []

        def longpoll():
            try:
                RPCProxy(n.rpcport, n.user, n.password).waitfornewblock(4000)
                results.append("ok")
            except RPCError as e:
                results.append(e.message)
            except Exception as e:  # the 500 reply carries no JSON body
                results.append(str(e))

        ts = [threading.Thread(target=longpoll) for _ in range(2)]
        for t in ts:
            t.start()
        time.sleep(1.0)  # both long polls are in flight: the queue is full
        import base64
        import http.client
        c = http.client.HTTPConnection("127.0.0.1", n.rpcport, timeout=30)
        auth = base64.b64encode(f"{n.user}:{n.password}".encode()).decode()
        c.request("POST", "/", body='{"method":"getblockcount","params":[],"id":1}',
                  headers={"Authorization": "Basic " + auth, "Content-Type": "application/json"})
        r = c.getresponse()
        assert r.status == 500 and r.read() == b"Work queue depth exceeded"
        c.close()
        for t in ts:
            t.join()
        assert results == ["ok", "ok"]
        assert n.rpc.getblockcount() == 1  # served again once the long polls are done
        assert "request rejected because http work queue depth exceeded" in debug_log(n)
    finally:
        n.stop()


def test_mocktime_and_stopafterblockimport(tmp_path):
    mock = 1700000000
    n = node(tmp_path, "n", f"-mocktime={mock}")
    try:
        h = n.rpc.generate(3)
        assert n.rpc.getblockheader(h[0])["time"] == mock + 1 or n.rpc.getblockheader(h[0])["time"] == mock
    finally:
        n.stop()
    # -loadblock the blocks of that chain into a fresh node with -stopafterblockimport
    blk = os.path.join(n.datadir, "regtest", "blocks", "blk00000.dat")
    code, out, m = run_to_exit(tmp_path, "m", f"-loadblock={blk}", "-stopafterblockimport", f"-mocktime={mock}")
    assert code == 0, out
    log = debug_log(m)
    assert "Stopping after block import" in log
    assert "height=3" in log


@pytest.mark.parametrize("arg,msg", [
    ("-socks=5", "Unsupported argument -socks found. Setting SOCKS version isn't possible anymore"),
    ("-tor=1", "Unsupported argument -tor found, use -onion."),
    ("-rpcssl=1", "SSL mode for RPC (-rpcssl) is no longer supported."),
])
def test_obsolete_options_refused(tmp_path, arg, msg):
    code, out, n = run_to_exit(tmp_path, "n" + arg[1:4], arg)
    assert code != 0
    assert msg in out or msg in debug_log(n)


def test_obsolete_options_warned(tmp_path):
    n = node(tmp_path, "n", "-benchmark", "-debugnet", "-blockminsize=1000", "-whitelistalwaysrelay")
    try:
        n.rpc.getblockcount()
        log = debug_log(n) + n.tail_log(20000)
        for w in ("Unsupported argument -benchmark ignored, use -debug=bench.",
                  "Unsupported argument -debugnet ignored, use -debug=net.",
                  "Unsupported argument -blockminsize ignored.",
                  "Unsupported argument -whitelistalwaysrelay ignored"):
            assert w in log, w
    finally:
        n.stop()


def test_sysperms(tmp_path):
    n = node(tmp_path, "n")
    try:
        mode = stat.S_IMODE(os.stat(os.path.join(n.datadir, "regtest", "debug.log")).st_mode)
        assert mode & 0o077 == 0, oct(mode)
    finally:
        n.stop()
    old = os.umask(0o022)
    try:
        m = node(tmp_path, "m", "-sysperms", "-disablewallet")
        try:
            mode = stat.S_IMODE(os.stat(os.path.join(m.datadir, "regtest", "debug.log")).st_mode)
            assert mode & 0o044 == 0o044, oct(mode)
        finally:
            m.stop()
        code, out, w = run_to_exit(tmp_path, "w", "-sysperms")
        assert code != 0
        assert "-sysperms is not allowed in combination with enabled wallet functionality" in out + debug_log(w)
    finally:
        os.umask(old)


def test_wallet_versions_and_upgradewallet(tmp_path):
    n = node(tmp_path, "hd")
    try:
        assert n.rpc.getwalletinfo()["walletversion"] == 130000
    finally:
        n.stop()
    code, out, _ = run_to_exit(tmp_path, "hd", "-upgradewallet=60000")
    assert code != 0 and "Cannot downgrade wallet" in out
    m = node(tmp_path, "plain", "-usehd=0")
    try:
        assert m.rpc.getwalletinfo()["walletversion"] == 60000
    finally:
        m.stop()
    # a store written by a newer client is refused
    code, out, _ = run_to_exit(tmp_path, "free", "-sendfreetransactions")
    assert code != 0 and "Creation of free transactions with their relay disabled is not supported." in out


def test_walletrejectlongchains(tmp_path):
    n = node(tmp_path, "n", "-walletrejectlongchains", "-limitancestorcount=5", "-limitdescendantcount=5")
    try:
        n.rpc.generate(101)
        addr = n.rpc.getnewaddress()
        # one coin, spent to ourselves over and over: each send chains on the previous change
        sent = 0
        with pytest.raises(RPCError) as e:
            for _ in range(10):
                n.rpc.sendtoaddress(addr, 1)
                sent += 1
        assert "Transaction has too long of a mempool chain" in e.value.message
        assert sent == 5  # a sixth would make a chain of 6 > -limitancestorcount=5
    finally:
        n.stop()


def test_printpriority_helpdebug_dns(tmp_path):
    n = node(tmp_path, "n", "-printpriority")
    try:
        n.rpc.generate(101)
        txid = n.rpc.sendtoaddress(n.rpc.getnewaddress(), 1)
        n.rpc.generate(1)
        assert any(l.startswith("priority") or " priority " in l and txid in l
                   for l in debug_log(n).splitlines() if txid in l)
    finally:
        n.stop()
    help_ = subprocess.run([os.path.join(BIN_DIR, "bcpd"), "-help", "-help-debug"], capture_output=True, text=True).stdout
    for opt in ("-mocktime", "-stopafterblockimport", "-printpriority", "-walletrejectlongchains", "-flushwallet"):
        assert opt in help_
    assert "-mocktime" not in subprocess.run([os.path.join(BIN_DIR, "bcpd"), "-help"], capture_output=True,
                                             text=True).stdout
    a = node(tmp_path, "a")
    b = node(tmp_path, "b", "-dns=0")
    try:
        b.rpc.addnode(f"localhost:{a.p2p_port}", "onetry")
        time.sleep(1.5)
        assert b.rpc.getconnectioncount() == 0  # the name is never resolved
        b.rpc.addnode(f"127.0.0.1:{a.p2p_port}", "onetry")
        assert wait_until(lambda: b.rpc.getconnectioncount() == 1)
    finally:
        a.stop()
        b.stop()
