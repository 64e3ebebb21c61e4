"""Browser wallet GUI (-webgui, csrc/rpc/webgui.cpp), the stand-in for the reference's Qt wallet
(src/qt/): served at GET /gui to authenticated RPC users only; every RPC method and result
field the page uses exists on this node; and the page's own script, run by node against a live
node, renders every tab and performs every action (test_webgui_page_script_drives_the_node)."""
import base64
import http.client
import json
import os
import re
import shutil
import subprocess

import pytest

from bitcoincashplus_amd.node.process import BcpdProcess

pytestmark = pytest.mark.functional


def _get(port, path, auth=None, method="GET", headers=None, body=None):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
    h = dict(headers or {})
    if auth:
        h["Authorization"] = "Basic " + base64.b64encode(auth.encode()).decode()
    c.request(method, path, body=body, headers=h)
    r = c.getresponse()
    body = r.read()
    return r.status, dict(r.getheaders()), body


def test_webgui(tmp_path):
    n = BcpdProcess(str(tmp_path / "g"), extra_args=["-gpu=0", "-webgui=1"])
    n.start()
    try:
        st, hdr, _ = _get(n.rpcport, "/gui")
        assert st == 401 and "Basic" in hdr.get("WWW-Authenticate", "")
        st, _, _ = _get(n.rpcport, "/gui", auth="rt:wrong")
        assert st == 401
        st, _, _ = _get(n.rpcport, "/gui", auth="rt:rtpass", method="POST")
        assert st == 405
        st, hdr, body = _get(n.rpcport, "/gui", auth="rt:rtpass")
        assert st == 200 and hdr["Content-Type"].startswith("text/html")
        page = body.decode()
        assert "<title>Bitcoin Cash Plus wallet</title>" in page

        # every method the page calls is registered (help errors on unknown commands)
        methods = set(re.findall(r'rpc\("([a-z]+)"', page))
        assert {"getbalance", "sendtoaddress", "getnewaddress", "listtransactions", "getpeerinfo",
                "getmininginfo", "generate", "decodepaymentrequest", "sendpaymentrequest", "execconsole", "parsebitcoinuri", "formatbitcoinuri", "signmessage", "verifymessage", "sendwithcoincontrol", "listunspent"} <= methods
        for m in sorted(methods):
            assert m in n.rpc.help(m), m

        # the result fields the page reads
        n.rpc.generate(101)
        addr = n.rpc.getnewaddress("gui")
        txid = n.rpc.sendtoaddress(addr, 1.5)
        bc = n.rpc.getblockchaininfo()
        for k in ("chain", "blocks", "headers", "bestblockhash", "difficulty", "verificationprogress"):
            assert k in bc, k
        net = n.rpc.getnetworkinfo()
        assert "connections" in net and "subversion" in net
        assert "immature_balance" in n.rpc.getwalletinfo()
        n.rpc.getunconfirmedbalance()
        txs = n.rpc.listtransactions("*", 10)
        assert any(t.get("txid") == txid for t in txs)
        for t in txs:
            for k in ("category", "amount", "confirmations", "time"):
                assert k in t, k
        rcv = n.rpc.listreceivedbyaddress(0, True)
        assert any(r["address"] == addr for r in rcv)
        for r in rcv:
            assert "amount" in r and "confirmations" in r and ("label" in r or "account" in r)
        mi = n.rpc.getmininginfo()
        assert "blocks" in mi and "difficulty" in mi
        assert isinstance(n.rpc.getgpuinfo(), dict)
        assert isinstance(n.rpc.getpeerinfo(), list)

        # the Qt-parity pages: address book, several recipients, payment requests, fees,
        # traffic, banned peers, backup, encryption
        assert {"sendmany", "setaccount", "listaddressgroupings", "getmempoolinfo", "uptime", "getnettotals",
                "listbanned", "setban", "clearbanned", "estimatesmartfee", "settxfee", "backupwallet",
                "encryptwallet", "walletpassphrasechange", "walletlock"} <= methods
        mp = n.rpc.getmempoolinfo()
        assert "size" in mp and "bytes" in mp and mp["size"] >= 1
        assert isinstance(n.rpc.uptime(), int)
        n.rpc.setaccount(addr, "relabelled")
        assert any(r["address"] == addr and (r.get("label") or r.get("account")) == "relabelled"
                   for r in n.rpc.listreceivedbyaddress(0, True))
        groups = n.rpc.listaddressgroupings()
        assert groups and all(isinstance(g[0], str) and len(g) >= 2 for grp in groups for g in grp)
        a2, a3 = n.rpc.getnewaddress(), n.rpc.getnewaddress()
        many = n.rpc.sendmany("", {a2: 0.25, a3: 0.5}, 1, "gui", [a2, a3])
        assert len(many) == 64
        uri = n.rpc.formatbitcoinuri(a2, 0.1, "lbl", "for tea")
        assert uri.endswith("amount=0.10000000&label=lbl&message=for%20tea") or "message=for" in uri
        ef = n.rpc.estimatesmartfee(6)
        assert "feerate" in ef and "blocks" in ef
        n.rpc.settxfee(0.0002)
        assert abs(n.rpc.getwalletinfo()["paytxfee"] - 0.0002) < 1e-12
        nt = n.rpc.getnettotals()
        assert "totalbytesrecv" in nt and "totalbytessent" in nt
        n.rpc.setban("192.0.2.7", "add", 86400)
        bans = n.rpc.listbanned()
        assert any(b["address"].startswith("192.0.2.7") and "banned_until" in b for b in bans)
        n.rpc.setban(bans[0]["address"], "remove")
        assert n.rpc.listbanned() == []
        n.rpc.setban("192.0.2.8", "add", 86400)
        n.rpc.clearbanned()
        assert n.rpc.listbanned() == []
        bk = tmp_path / "gui-backup"
        n.rpc.backupwallet(str(bk))
        assert bk.exists()
        assert "unlocked_until" not in n.rpc.getwalletinfo()
        n.rpc.encryptwallet("pass one")
        wi = n.rpc.getwalletinfo()
        assert wi["unlocked_until"] == 0
        n.rpc.walletpassphrasechange("pass one", "pass two")
        n.rpc.walletpassphrase("pass two", 60)
        assert n.rpc.getwalletinfo()["unlocked_until"] > 0
        n.rpc.walletlock()
        assert n.rpc.getwalletinfo()["unlocked_until"] == 0
    finally:
        n.stop()

    # the page is off by default
    m = BcpdProcess(str(tmp_path / "h"), extra_args=["-gpu=0"])
    m.start()
    try:
        st, _, _ = _get(m.rpcport, "/gui", auth="rt:rtpass")
        assert st == 404
    finally:
        m.stop()


def test_rpc_refuses_cross_site_browser_requests(tmp_path):
    """A browser on another site may hold Basic credentials cached for the GUI: a cross-origin
    "simple" POST (text/plain, no custom header) must not reach the RPC table, while the GUI's
    own same-origin JSON request and non-browser clients (no Origin) are served."""
    n = BcpdProcess(str(tmp_path / "c"), extra_args=["-gpu=0", "-webgui=1"])
    n.start()
    try:
        body = '{"method":"getblockcount","params":[],"id":1}'
        host = f"127.0.0.1:{n.rpcport}"
        cases = [
            ({"Origin": "http://evil.example", "Content-Type": "text/plain"}, 403),
            ({"Origin": "http://evil.example", "Content-Type": "application/json",
              "X-Requested-With": "x"}, 403),
            ({"Origin": "http://" + host, "Content-Type": "text/plain", "X-Requested-With": "x"}, 403),
            ({"Origin": "http://" + host, "Content-Type": "application/json"}, 403),
            ({"Origin": "null", "Content-Type": "application/json", "X-Requested-With": "x"}, 403),
            ({"Origin": "http://" + host, "Content-Type": "application/json",
              "X-Requested-With": "bcp-webgui"}, 200),
            ({"Content-Type": "text/plain"}, 200),  # curl / bcp-cli style, no Origin
        ]
        for hdr, want in cases:
            st, _, out = _get(n.rpcport, "/", auth="rt:rtpass", method="POST", headers=hdr, body=body)
            assert st == want, (hdr, st, out)
            if want == 200:
                assert b'"result":0' in out.replace(b" ", b"")
    finally:
        n.stop()


@pytest.mark.skipif(shutil.which("node") is None, reason="no JavaScript engine (node) on this host")
def test_webgui_page_script_drives_the_node(tmp_path):
    """The page's own JavaScript, run by node against a live bcpd through a minimal DOM
    (tests/data/webgui_driver.js): every tab renders without an RPC error, and every action -
    generate, payment request, send to one and to several recipients, label edit, fee, backup,
    encryption, passphrase change, lock and the passphrase prompt, ban/unban, sign/verify and the
    console - goes through the page's functions."""
    n = BcpdProcess(str(tmp_path / "g"), extra_args=["-gpu=0", "-webgui=1"])
    n.start()
    try:
        st, _, body = _get(n.rpcport, "/gui", auth="rt:rtpass")
        assert st == 200
        page = body.decode()
        script = page[page.index("<script>") + len("<script>"):page.index("</script>")]
        js = tmp_path / "page.js"
        js.write_text(script)
        chk = subprocess.run(["node", "--check", str(js)], capture_output=True, text=True)
        assert chk.returncode == 0, chk.stderr
        bk = tmp_path / "gui-backup.dat"
        drv = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "webgui_driver.js")
        r = subprocess.run(["node", drv, str(js), str(n.rpcport), "rt:rtpass", str(bk)], capture_output=True,
                           text=True, timeout=240)
        out = json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else {"error": r.stderr[-2000:]}
        assert r.returncode == 0 and out.get("ok"), out
        assert out["encstate_before"] == "not encrypted" and out["encstate_after"] == "encrypted, locked"
        assert "received_bytes" in out["traffic"]
        assert bk.exists()
        assert n.rpc.getaccount(out["request_uri"].split(":", 1)[1].split("?")[0]) == "renamed"
    finally:
        n.stop()
