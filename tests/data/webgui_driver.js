// Runs the web GUI page's script (csrc/rpc/webgui.cpp) against a live bcpd with a minimal DOM:
// node webgui_driver.js PAGE_SCRIPT.js RPCPORT USER:PASS BACKUP_PATH
// Every tab is refreshed and every page action is invoked through the page's own functions;
// prints one JSON object with what the page rendered, exits non-zero on the first failure.
"use strict";
const fs = require("fs");
const http = require("http");
const vm = require("vm");

const [script, port, auth, backupPath] = process.argv.slice(2);

function makeEl(id) {
  const el = {
    id, textContent: "", innerHTML: "", value: "", checked: false, style: {}, dataset: {}, children: [],
    listeners: {},
    classList: { set: new Set(), toggle(c, on) { on ? this.set.add(c) : this.set.delete(c); }, add(c) { this.set.add(c); } },
    addEventListener(ev, fn) { this.listeners[ev] = fn; },
    appendChild(c) { this.children.push(c); },
    querySelector(sel) { return this.sub ? this.sub[sel] : null; },
    click() {},
    set scrollTop(v) {},
  };
  return el;
}
const els = {};
const document = {
  getElementById(id) { return els[id] || (els[id] = makeEl(id)); },
  createElement(tag) { return makeEl("<" + tag + ">"); },
  querySelectorAll(sel) {
    if (sel === ".rcp") return els["morercp"] ? els["morercp"].children : [];
    return [];
  },
};
const store = {};
const localStorage = {
  getItem: k => (k in store ? store[k] : null), setItem: (k, v) => { store[k] = String(v); }, removeItem: k => { delete store[k]; },
};

function fetch(url, opts) {
  return new Promise((resolve, reject) => {
    const req = http.request({ host: "127.0.0.1", port: Number(port), path: "/", method: "POST",
      headers: { "Content-Type": "application/json", Authorization: "Basic " + Buffer.from(auth).toString("base64") } }, res => {
      let body = "";
      res.on("data", d => { body += d; });
      res.on("end", () => resolve({ json: async () => JSON.parse(body) }));
    });
    req.on("error", reject);
    req.end(opts.body);
  });
}

const ctx = vm.createContext({
  document, localStorage, fetch, console, JSON, Promise, Object, Number, String, Math, Date, Buffer,
  setInterval: () => 0, alert: m => { throw new Error("alert: " + m); },
  URL: { createObjectURL: () => "blob:" }, Blob: function () {},
});
vm.runInContext(fs.readFileSync(script, "utf8"), ctx);

const $ = id => document.getElementById(id);
const out = {};
function fail(msg) { console.log(JSON.stringify(Object.assign(out, { error: msg }))); process.exit(1); }
async function call(expr) { return vm.runInContext(expr, ctx); }
async function tab(name) {
  $("status").innerHTML = "";
  await call(`refresh(${JSON.stringify(name)})`);
  if ($("status").innerHTML.includes("err")) fail(name + ": " + $("status").innerHTML);
}

(async () => {
  await tab("mining");
  $("gencount").value = "101";
  await call("doGenerate()");
  if (!$("genres").innerHTML.includes("101 block(s)")) fail("generate: " + $("genres").innerHTML);
  for (const t of ["overview", "send", "receive", "transactions", "addresses", "wallet", "signverify", "peers", "mining", "console"])
    await tab(t);
  out.balance = $("bal").textContent;
  out.status = $("status").textContent;

  // receive: a payment request with amount and message, kept in the requested-payments table
  $("rcvlabel").value = "tea"; $("rcvamt").value = "0.5"; $("rcvmsg").value = "for tea";
  await call("newAddr()");
  out.request_uri = $("newaddr").textContent;
  if (!/amount=0\.5/.test(out.request_uri) || !/message=for/.test(out.request_uri)) fail("request: " + out.request_uri);
  await tab("receive");
  if (!$("reqlist").innerHTML.includes("for tea")) fail("requested payments table");
  const addr = out.request_uri.replace(/^[a-z]+:/, "").split("?")[0];

  // send to one recipient, then to two (sendmany)
  $("sendto").value = addr; $("sendamt").value = "1";
  await call("doSend()");
  if (!$("sendres").innerHTML.includes("sent ")) fail("send: " + $("sendres").innerHTML);
  await call("addRcp()");
  const extra = $("morercp").children[0];
  extra.sub = { ".rto": { value: addr }, ".ramt": { value: "0.25" } };
  const other = await call("rpc('getnewaddress')");
  $("sendto").value = other;
  await call("doSend()");
  out.sendmany = $("sendres").innerHTML;
  if (!out.sendmany.includes("2 recipients")) fail("sendmany: " + out.sendmany);

  // address book: edit a label
  await tab("addresses");
  if (!$("ablist").innerHTML.includes(addr)) fail("address book misses " + addr);
  $("lblx").value = "renamed";
  await call(`setLabel(${JSON.stringify(addr)}, "lblx")`);
  const acct = await call(`rpc("getaccount", [${JSON.stringify(addr)}])`);
  if (acct !== "renamed") fail("label not saved: " + acct);
  if (!$("grplist").innerHTML.includes("BCP")) fail("address groupings empty");

  // wallet: fee, backup, encryption, passphrase change, lock
  await tab("wallet");
  out.encstate_before = $("encstate").textContent;
  $("feerate").value = "0.0003";
  await call("setFee()");
  if (!$("feeres").innerHTML.includes("set")) fail("fee: " + $("feeres").innerHTML);
  $("bkpath").value = backupPath;
  await call("backupWallet()");
  if (!$("bkres").innerHTML.includes("backed up")) fail("backup: " + $("bkres").innerHTML);
  $("encpass1").value = "a"; $("encpass2").value = "b";
  await call("encryptWallet()");
  if (!$("encres").innerHTML.includes("differ")) fail("mismatched passphrases accepted");
  $("encpass1").value = "gui pass"; $("encpass2").value = "gui pass";
  await call("encryptWallet()");
  if (!$("encres").innerHTML.includes("ok")) fail("encrypt: " + $("encres").innerHTML);
  await tab("wallet");
  out.encstate_after = $("encstate").textContent;
  $("chgold").value = "gui pass"; $("chgnew1").value = "gui pass 2"; $("chgnew2").value = "gui pass 2";
  await call("changePass()");
  if (!$("encres").innerHTML.includes("passphrase changed")) fail("change: " + $("encres").innerHTML);
  await call("lockWallet()");

  // a locked wallet asks for the passphrase on send, and the send goes through with it
  $("sendto").value = addr; $("sendamt").value = "0.1"; $("morercp").children = [];
  await call("doSend()");
  if ($("passrow").style.display !== "block") fail("no passphrase prompt for a locked wallet");
  $("sendpass").value = "gui pass 2";
  await call("doSend()");
  if (!$("sendres").innerHTML.includes("sent ")) fail("send after unlock: " + $("sendres").innerHTML);

  // peers: traffic totals, ban and unban
  await call('banPeer("192.0.2.9:8333")');
  await tab("peers");
  out.traffic = $("traffic").innerHTML;
  if (!$("banlist").innerHTML.includes("192.0.2.9")) fail("ban not listed");
  const ban = (await call('rpc("listbanned")')).find(x => x.address.includes("192.0.2.9"));
  await call(`unban(${JSON.stringify(ban.address)})`);
  await tab("peers");
  if ($("banlist").innerHTML.includes("192.0.2.9")) fail("unban");

  // sign / verify
  $("smaddr").value = addr; $("smmsg").value = "hello";
  $("sendpass").value = "gui pass 2";
  await call("signMsg()");
  $("vmaddr").value = addr; $("vmmsg").value = "hello"; $("vmsig").value = $("smsig").textContent;
  await call("verifyMsg()");
  if (!$("vmres").innerHTML.includes("message verified")) fail("verify: " + $("vmres").innerHTML);

  // console: one command, through the page's key handler
  $("conin").value = "getblockcount";
  await $("conin").listeners.keydown({ key: "Enter" });
  out.console = $("conout").textContent;
  if (!/> getblockcount\n\d+/.test(out.console)) fail("console: " + out.console);

  out.ok = true;
  console.log(JSON.stringify(out));
})().catch(e => fail(String(e && (e.stack || e.message) || e)));
