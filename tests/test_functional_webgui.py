"""Browser wallet GUI (-webgui, csrc/rpc/webgui.cpp), the stand-in for the reference's Qt wallet
(src/qt/): served at GET /gui to authenticated RPC users only, and every RPC method and result
field the page uses exists on this node (the page's JavaScript is not executed here)."""
import base64
import http.client
import re

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
