"""RPC console command lines (csrc/rpc/console.{h,cpp}, RPC `execconsole`).

Parity: reference src/qt/test/rpcnestedtests.cpp, which runs RPCConsole::RPCExecuteCommandLine
and RPCParseCommandLine against a node. The same lines run here through `console_parse` with a
Python executor (its `rpcNestedTest` echoes the argument list as JSON text, like the reference's
test-only RPC) and through `execconsole` on a regtest node for the nested chain calls.
"""
import json

import pytest

from bitcoincashplus_amd import native


def echo_exec(method, args):
    if method == "rpcNestedTest":
        return json.dumps(json.dumps(args, separators=(",", ":")))  # a string result
    if method == "getblockchaininfo":
        return json.dumps({"chain": "main", "blocks": 0})
    if method == "getbestblockhash":
        return json.dumps("00ab")
    if method == "getblock":
        assert args == ["00ab"]
        return json.dumps({"hash": "00ab", "tx": ["4a5e1e", "ffee"]})
    raise RuntimeError(f"method not found: {method}")


def run(line):
    return native.console_parse(line, echo_exec)[0]


def filtered(line):
    return native.console_parse(line)[1]


def test_nested_calls_and_queries():
    assert run("getblockchaininfo()[chain]") == "main"
    assert native.console_parse("getblockchaininfo()[chain]", echo_exec)[1] == "getblockchaininfo()[chain]"
    assert run("getblock(getbestblockhash())[tx][0]") == "4a5e1e"
    assert run("getblock(getbestblockhash())[tx][5]") == "null"
    assert run("getblockchaininfo").startswith("{")
    assert run("getblockchaininfo()").startswith("{")
    assert run("getblockchaininfo ").startswith("{")
    assert run("getblockchaininfo()[nonexistent]") == "null"
    with pytest.raises(RuntimeError, match="Invalid result query"):
        run("getblock(getbestblockhash())[tx][x]")
    with pytest.raises(RuntimeError, match="Invalid result query"):
        run("getbestblockhash()[0]")


def test_argument_splitting():
    assert run("rpcNestedTest") == "[]"
    assert run("rpcNestedTest ''") == '[""]'
    assert run('rpcNestedTest ""') == '[""]'
    assert run("rpcNestedTest '' abc") == '["","abc"]'
    assert run("rpcNestedTest abc '' abc") == '["abc","","abc"]'
    assert run("rpcNestedTest abc  abc") == '["abc","abc"]'
    assert run("rpcNestedTest abc\t\tabc") == '["abc","abc"]'
    assert run("rpcNestedTest(abc )") == '["abc"]'
    assert run("rpcNestedTest( abc )") == '["abc"]'
    assert run("rpcNestedTest(   abc   ,   cba )") == '["abc","cba"]'
    assert run("rpcNestedTest [] {} 0") == run("rpcNestedTest( [],  {} , 0   )") == '["[]","{}","0"]'
    # quoting and escapes
    assert run(r'rpcNestedTest "a \"q\" \\ \n" \x') == json.dumps(['a "q" \\ \\n', "x"], separators=(",", ":"))
    assert run("rpcNestedTest 'a \\ \" b'") == json.dumps(['a \\ " b'], separators=(",", ":"))
    # a nested call's string result becomes one argument
    assert run("rpcNestedTest(getbestblockhash(), x)") == '["00ab","x"]'


def test_syntax_errors():
    for bad in ("getblockchaininfo() .\n", "getblockchaininfo() getblockchaininfo()", "rpcNestedTest abc,,abc",
                "rpcNestedTest(abc,,abc)", "rpcNestedTest(abc,,)", "rpcNestedTest 'abc"):
        with pytest.raises(RuntimeError):
            run(bad)
    run("getblockchaininfo(")        # an unclosed bracket without arguments is tolerated
    run("getblockchaininfo()()()")   # as are stray brackets after the call
    with pytest.raises(RuntimeError, match="method not found"):
        run("a(getblockchaininfo(True))")


def test_hostile_lines():
    """Deep nesting is a syntax error, not a stack overflow (with or without execution), and an
    array index longer than any array is out of range, not an uncaught std::out_of_range."""
    deep = "a(" * 100000
    with pytest.raises(RuntimeError, match="Invalid Syntax"):
        run(deep)
    with pytest.raises(RuntimeError, match="Invalid Syntax"):
        native.console_parse(deep)
    assert run("getbestblockhash(" * 60 + ")" * 60) == "00ab"  # 60 levels are still fine
    assert run("getblock(getbestblockhash())[tx][99999999999999999999]") == "null"
    assert run("getblock(getbestblockhash())[tx][1]") == "ffee"


def test_history_filter():
    assert filtered("importprivkey") == "importprivkey(…)"
    assert filtered("signmessagewithprivkey abc") == "signmessagewithprivkey(…)"
    assert filtered("signmessagewithprivkey abc,def") == "signmessagewithprivkey(…)"
    assert filtered("signrawtransaction(abc)") == "signrawtransaction(…)"
    assert filtered("walletpassphrase(help())") == "walletpassphrase(…)"
    assert filtered("walletpassphrasechange(help(walletpassphrasechange(abc)))") == "walletpassphrasechange(…)"
    assert filtered("help(encryptwallet(abc, def))") == "help(encryptwallet(…))"
    assert filtered("help(importprivkey())") == "help(importprivkey(…))"
    assert filtered("help(importprivkey(help()))") == "help(importprivkey(…))"
    assert filtered("help(importprivkey(abc), walletpassphrase(def))") == "help(importprivkey(…), walletpassphrase(…))"
    assert filtered("getblock(getbestblockhash())[tx][0]") == "getblock(getbestblockhash())[tx][0]"


@pytest.mark.functional
def test_execconsole_on_node(tmp_path):
    from bitcoincashplus_amd.node.embedded import RPCError
    from bitcoincashplus_amd.node.process import BcpdProcess

    n = BcpdProcess(str(tmp_path / "n"), extra_args=["-gpu=0", "-keypool=5"])
    n.start()
    try:
        n.rpc.generate(3)
        r = n.rpc.execconsole("getblock(getbestblockhash())[tx][0]")
        best = n.rpc.getblock(n.rpc.getbestblockhash())
        assert r["result"] == best["tx"][0]
        assert n.rpc.execconsole("getblockchaininfo()[chain]")["result"] == "regtest"
        assert n.rpc.execconsole("getblockcount")["result"] == "3"
        addr = n.rpc.getnewaddress()
        assert n.rpc.execconsole(f"validateaddress({addr})[isvalid]")["result"] == "true"
        assert n.rpc.execconsole("validateaddress(getnewaddress())[ismine]")["result"] == "true"
        assert n.rpc.execconsole("createrawtransaction [] {} 0")["result"] == \
            n.rpc.execconsole("createrawtransaction( [],  {} , 0   )")["result"]
        with pytest.raises(RPCError):
            n.rpc.execconsole("getblockchaininfo() getblockchaininfo()")
        with pytest.raises(RPCError):
            n.rpc.execconsole("a(getblockcount())")
        with pytest.raises(RPCError) as e:
            n.rpc.execconsole("importprivkey(notakey)")
        assert e.value.code != 0
    finally:
        n.stop()
