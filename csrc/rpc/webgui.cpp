// Browser wallet GUI served by bcpd (GET /gui on the RPC port, -webgui).
// Parity: reference src/qt/ (bitcoin-qt: overview page with balances and recent transactions,
// send coins dialog, receive coins with labels, transaction list, peers table, debug console
// with RPC history). Qt is not available here; the same functions are a single page that
// talks JSON-RPC to this node over the authenticated HTTP port, so it needs no extra
// dependency and no separate binary. The page is served only to authenticated RPC users.
#include "rpc/httpserver.h"
#include "util/strencodings.h"
#include "util/util.h"

namespace bcp {

static const char* const kGuiPage = R"BCPGUI(<!DOCTYPE html>
<html lang="en"><head><meta charset="utf-8"><title>Bitcoin Cash Plus wallet</title>
<meta name="viewport" content="width=device-width, initial-scale=1">
<style>
body{font-family:system-ui,sans-serif;margin:0;background:#f4f5f7;color:#222}
header{background:#1d3557;color:#fff;padding:10px 18px;display:flex;align-items:center;gap:18px}
header h1{font-size:18px;margin:0}nav button{background:none;border:0;color:#cfd8e3;font-size:15px;padding:6px 10px;cursor:pointer}
nav button.on{color:#fff;border-bottom:2px solid #e63946}main{padding:18px;max-width:1100px}
section{display:none}section.on{display:block}.card{background:#fff;border-radius:6px;padding:14px 18px;margin-bottom:14px;box-shadow:0 1px 2px #0002}
table{border-collapse:collapse;width:100%;font-size:13px}td,th{padding:5px 8px;border-bottom:1px solid #eee;text-align:left;vertical-align:top}
.big{font-size:26px;font-weight:600}.mono{font-family:ui-monospace,monospace;word-break:break-all}
input,select{padding:6px;font-size:14px;margin:3px 0}input.wide{width:100%;box-sizing:border-box}
button.act{background:#1d3557;color:#fff;border:0;border-radius:4px;padding:7px 14px;cursor:pointer}
#status{margin-left:auto;font-size:13px;color:#cfd8e3}.err{color:#c1121f}.ok{color:#2a9d8f}
#conout{background:#111;color:#ddd;height:360px;overflow:auto;padding:8px;font-size:12px;white-space:pre-wrap}
</style></head><body>
<header><h1>Bitcoin Cash Plus</h1><nav id="tabs"></nav><span id="status">connecting…</span></header>
<main>
<section id="overview"><div class="card"><div>Available</div><div class="big" id="bal">–</div>
<div>Pending <span id="ubal">–</span> · Immature <span id="ibal">–</span></div></div>
<div class="card"><table><tbody id="chaininfo"></tbody></table></div>
<div class="card"><b>Recent transactions</b><table><thead><tr><th>Date</th><th>Type</th><th>Address</th><th>Amount</th><th>Conf.</th></tr></thead><tbody id="recent"></tbody></table></div></section>
<section id="send"><div class="card"><div>Pay to</div><input class="wide" id="sendto" placeholder="address (CashAddr or Base58)">
<div>Amount (BCP)</div><input id="sendamt" type="number" step="0.00000001" min="0">
<label><input type="checkbox" id="sendsub"> subtract fee from amount</label>
<div>Comment</div><input class="wide" id="sendcomment">
<div id="passrow" style="display:none">Wallet passphrase <input type="password" id="sendpass"></div>
<p><button class="act" onclick="doSend()">Send</button> <span id="sendres"></span></p>
<details id="cc"><summary>Coin control</summary><p><button onclick="loadCoins()">List coins</button> Change address <input class="wide" id="ccchange"></p>
<table><thead><tr><th></th><th>Amount</th><th>Address</th><th>Conf.</th><th>Output</th></tr></thead><tbody id="cclist"></tbody></table></details></div>
<div class="card"><div>BIP70 payment request (hex or base64)</div><textarea class="wide" id="preq" rows="3"></textarea>
<p><button onclick="checkReq()">Check</button> <button class="act" onclick="payReq()">Pay request</button> <span id="preqres"></span></p>
<div id="preqinfo"></div></div></section>
<section id="receive"><div class="card">Label <input id="rcvlabel"> <button class="act" onclick="newAddr()">New address</button>
<p class="mono big" id="newaddr"></p></div>
<div class="card"><b>Receiving addresses</b><table><thead><tr><th>Address</th><th>Label</th><th>Received</th><th>Conf.</th></tr></thead><tbody id="rcvlist"></tbody></table></div></section>
<section id="transactions"><div class="card"><button onclick="exportCsv()">Export CSV</button></div><div class="card"><table><thead><tr><th>Date</th><th>Type</th><th>Address</th><th>Amount</th><th>Conf.</th><th>Txid</th></tr></thead><tbody id="txlist"></tbody></table></div></section>
<section id="signverify"><div class="card"><b>Sign message</b><div>Address</div><input class="wide" id="smaddr">
<div>Message</div><textarea class="wide" id="smmsg" rows="3"></textarea>
<p><button class="act" onclick="signMsg()">Sign</button></p><p class="mono" id="smsig"></p></div>
<div class="card"><b>Verify message</b><div>Address</div><input class="wide" id="vmaddr">
<div>Message</div><textarea class="wide" id="vmmsg" rows="3"></textarea><div>Signature</div><input class="wide" id="vmsig">
<p><button class="act" onclick="verifyMsg()">Verify</button> <span id="vmres"></span></p></div></section>
<section id="peers"><div class="card"><table><thead><tr><th>Address</th><th>Client</th><th>Version</th><th>Direction</th><th>Height</th><th>Sent</th><th>Recv</th><th>Ping ms</th></tr></thead><tbody id="peerlist"></tbody></table></div></section>
<section id="mining"><div class="card"><table><tbody id="mininfo"></tbody></table></div>
<div class="card"><table><tbody id="gpuinfo"></tbody></table></div>
<div class="card">Generate <input id="gencount" type="number" value="1" min="1" style="width:70px"> block(s) to this wallet (regtest)
<button class="act" onclick="doGenerate()">Generate</button> <span id="genres"></span></div></section>
<section id="console"><div class="card"><div id="conout"></div>
<input class="wide mono" id="conin" placeholder="method arg1 arg2 …  (e.g. getblockchaininfo, getblockhash 10; ↑/↓ history)"></div></section>
</main>
<script>
const TABS=[["overview","Overview"],["send","Send"],["receive","Receive"],["transactions","Transactions"],["signverify","Sign / verify"],["peers","Peers"],["mining","Mining"],["console","Console"]];
let rpcId=0;
async function rpc(method,params=[]){
  const r=await fetch("/",{method:"POST",credentials:"same-origin",headers:{"Content-Type":"application/json","X-Requested-With":"bcp-webgui"},
    body:JSON.stringify({jsonrpc:"1.0",id:++rpcId,method:method,params:params})});
  const j=await r.json(); if(j.error) throw j.error; return j.result;}
const $=id=>document.getElementById(id);
const esc=s=>String(s===undefined?"":s).replace(/[&<>"]/g,c=>({"&":"&amp;","<":"&lt;",">":"&gt;",'"':"&quot;"}[c]));
const amt=v=>(v===undefined?"–":Number(v).toFixed(8)+" BCP");
const date=t=>t?new Date(t*1000).toLocaleString():"";
function rows(tb,list,cols){$(tb).innerHTML=list.map(o=>"<tr>"+cols.map(c=>"<td class='"+(c[1]||"")+"'>"+esc(c[0](o))+"</td>").join("")+"</tr>").join("");}
function kv(tb,obj,keys){$(tb).innerHTML=keys.filter(k=>obj[k]!==undefined).map(k=>"<tr><th>"+esc(k)+"</th><td>"+esc(typeof obj[k]=="object"?JSON.stringify(obj[k]):obj[k])+"</td></tr>").join("");}
const TXCOLS=[[t=>date(t.time)],[t=>t.category],[t=>t.address||t.account||"",'mono'],[t=>amt(t.amount)],[t=>t.confirmations]];
function show(id){for(const [t] of TABS){$(t).classList.toggle("on",t==id);$("tab_"+t).classList.toggle("on",t==id);}refresh(id);}
$("tabs").innerHTML=TABS.map(([t,n])=>"<button id='tab_"+t+"' onclick=\"show('"+t+"')\">"+n+"</button>").join("");
let current="overview";
async function refresh(id){current=id||current;
  try{
    const bc=await rpc("getblockchaininfo");
    $("status").textContent=bc.chain+" · height "+bc.blocks+(bc.initialblockdownload?" · syncing":"");
    if(current=="overview"){
      const [b,u,w,n,tx]=await Promise.all([rpc("getbalance"),rpc("getunconfirmedbalance"),rpc("getwalletinfo"),rpc("getnetworkinfo"),rpc("listtransactions",["*",10])]);
      $("bal").textContent=amt(b);$("ubal").textContent=amt(u);$("ibal").textContent=amt(w.immature_balance);
      kv("chaininfo",Object.assign({},bc,{connections:n.connections,subversion:n.subversion}),["chain","blocks","headers","bestblockhash","difficulty","verificationprogress","connections","subversion"]);
      rows("recent",tx.reverse(),TXCOLS);}
    if(current=="receive") rows("rcvlist",await rpc("listreceivedbyaddress",[0,true]),[[a=>a.address,'mono'],[a=>a.label||a.account],[a=>amt(a.amount)],[a=>a.confirmations]]);
    if(current=="transactions") rows("txlist",(await rpc("listtransactions",["*",200])).reverse(),TXCOLS.concat([[t=>t.txid,'mono']]));
    if(current=="peers") rows("peerlist",await rpc("getpeerinfo"),[[p=>p.addr,'mono'],[p=>p.subver],[p=>p.version],[p=>p.inbound?"in":"out"],[p=>p.synced_blocks],[p=>p.bytessent],[p=>p.bytesrecv],[p=>p.pingtime===undefined?"":Math.round(p.pingtime*1000)]]);
    if(current=="mining"){
      kv("mininfo",await rpc("getmininginfo"),["blocks","difficulty","networkhashps","pooledtx","chain","errors"]);
      kv("gpuinfo",await rpc("getgpuinfo"),Object.keys(await rpc("getgpuinfo")));}
  }catch(e){$("status").innerHTML="<span class='err'>"+esc(e.message||e)+"</span>";}}
async function doSend(){
  $("sendres").textContent="";
  try{
    const to=$("sendto").value.trim();
    if(to.includes(":")&&to.includes("?")){const u=await rpc("parsebitcoinuri",[to]);$("sendto").value=u.address;
      if(u.amount>0)$("sendamt").value=u.amount; if(u.message)$("sendcomment").value=u.message;
      $("sendres").innerHTML="<span class='ok'>filled from URI — check and press Send</span>";return;}
    const pass=$("sendpass").value; if(pass) await rpc("walletpassphrase",[pass,60]);
    const picked=[...document.querySelectorAll(".ccpick:checked")].map(c=>({txid:c.dataset.txid,vout:Number(c.dataset.vout)}));
    if(picked.length){const to=$("sendto").value.trim(),amts={};amts[to]=Number($("sendamt").value);
      const r=await rpc("sendwithcoincontrol",[amts,picked,$("ccchange").value.trim(),$("sendsub").checked?[to]:[]]);
      $("sendres").innerHTML="<span class='ok'>sent "+esc(r.txid)+" (fee "+amt(r.fee)+")</span>";$("sendpass").value="";loadCoins();return;}
    const txid=await rpc("sendtoaddress",[$("sendto").value.trim(),Number($("sendamt").value),$("sendcomment").value,"",$("sendsub").checked]);
    $("sendres").innerHTML="<span class='ok'>sent "+esc(txid)+"</span>";$("sendpass").value="";
  }catch(e){ if(e.code==-13) $("passrow").style.display="block";
    $("sendres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function checkReq(){$("preqres").textContent="";
  try{const r=await rpc("decodepaymentrequest",[$("preq").value.trim()]);
    const who=r.merchant?"<span class='ok'>"+esc(r.merchant)+"</span>":"<span class='err'>unauthenticated"+(r.merchant_error?" ("+esc(r.merchant_error)+")":"")+"</span>";
    $("preqinfo").innerHTML="Merchant: "+who+"<br>Memo: "+esc(r.memo)+"<br>Pay: "+r.outputs.map(o=>esc(o.address||o.script)+" "+amt(o.amount)).join(", ")+
      (r.network_ok?"":"<br><span class='err'>network "+esc(r.network)+" does not match</span>")+(r.expired?"<br><span class='err'>expired</span>":"");
  }catch(e){$("preqres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function payReq(){$("preqres").textContent="";
  try{const pass=$("sendpass").value; if(pass) await rpc("walletpassphrase",[pass,60]);
    const r=await rpc("sendpaymentrequest",[$("preq").value.trim()]);
    $("preqres").innerHTML="<span class='ok'>paid "+esc(r.txid)+(r.payment_url?" (send the Payment to "+esc(r.payment_url)+")":"")+"</span>";
  }catch(e){ if(e.code==-13) $("passrow").style.display="block"; $("preqres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function signMsg(){try{const pass=$("sendpass").value; if(pass) await rpc("walletpassphrase",[pass,60]);
  $("smsig").textContent=await rpc("signmessage",[$("smaddr").value.trim(),$("smmsg").value]);}
  catch(e){$("smsig").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function verifyMsg(){try{const ok=await rpc("verifymessage",[$("vmaddr").value.trim(),$("vmsig").value.trim(),$("vmmsg").value]);
  $("vmres").innerHTML=ok?"<span class='ok'>message verified</span>":"<span class='err'>signature does not match</span>";}
  catch(e){$("vmres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function exportCsv(){const txs=await rpc("listtransactions",["*",100000]);
  const q=v=>'"'+String(v??"").replace(/"/g,'""')+'"';
  const lines=[["Confirmed","Date","Type","Label","Address","Amount","ID"].map(q).join(",")].concat(txs.map(t=>
    [t.confirmations>0,new Date(t.time*1000).toISOString(),t.category,t.label||t.account||"",t.address||"",t.amount,t.txid].map(q).join(",")));
  const a=document.createElement("a");a.href=URL.createObjectURL(new Blob([lines.join("\n")],{type:"text/csv"}));
  a.download="transactions.csv";a.click();}
async function loadCoins(){const u=await rpc("listunspent",[0]);
  $("cclist").innerHTML=u.map(c=>"<tr><td><input type='checkbox' class='ccpick' data-txid='"+esc(c.txid)+"' data-vout='"+c.vout+"'></td><td>"+amt(c.amount)+
    "</td><td class='mono'>"+esc(c.address||"")+"</td><td>"+c.confirmations+"</td><td class='mono'>"+esc(c.txid.slice(0,16))+"…:"+c.vout+"</td></tr>").join("");}
async function newAddr(){try{const a=await rpc("getnewaddress",[$("rcvlabel").value]);
  $("newaddr").textContent=a+"  "+await rpc("formatbitcoinuri",[a,null,$("rcvlabel").value]);refresh("receive");}
  catch(e){$("newaddr").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function doGenerate(){$("genres").textContent="mining…";
  try{const h=await rpc("generate",[Number($("gencount").value)]);$("genres").innerHTML="<span class='ok'>"+h.length+" block(s)</span>";refresh("mining");}
  catch(e){$("genres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
const hist=[];let hpos=0;
$("conin").addEventListener("keydown",async ev=>{
  if(ev.key=="ArrowUp"&&hpos>0){$("conin").value=hist[--hpos];return;}
  if(ev.key=="ArrowDown"&&hpos<hist.length){hpos++;$("conin").value=hist[hpos]||"";return;}
  if(ev.key!="Enter") return;
  const line=$("conin").value.trim(); if(!line) return; $("conin").value="";
  let text,shown=line;
  // the node parses the line (nested calls, [key] queries) and returns the history-safe form
  try{const r=await rpc("execconsole",[line]);text=r.result;shown=r.filtered;}catch(e){text="error "+e.code+": "+e.message;}
  // a line that failed to parse still keeps secrets out of the history
  if(/^(importprivkey|importmulti|signmessagewithprivkey|signrawtransaction|walletpassphrase|walletpassphrasechange|encryptwallet)\b/i.test(shown)&&shown==line) shown=shown.split(/[ (]/)[0]+"(…)";
  hist.push(shown);hpos=hist.length;
  $("conout").textContent+="> "+shown+"\n"+text+"\n\n";$("conout").scrollTop=1e9;});
show("overview");setInterval(()=>refresh(),5000);
</script></body></html>
)BCPGUI";

static bool HTTPReq_GUI(const HTTPRequest& req, HTTPReply& rep) {
    if (req.method != "GET") {
        rep.status = 405;
        rep.contentType = "text/plain";
        rep.body = "the wallet GUI handles only GET";
        return false;
    }
    std::string user;
    if (!RPCAuthorizedHeader(req.Header("authorization"), user)) {
        rep.status = 401;
        rep.contentType = "text/plain";
        rep.extraHeaders["WWW-Authenticate"] = "Basic realm=\"bcp-gui\"";
        rep.body = "authentication required (RPC credentials)";
        return false;
    }
    rep.status = 200;
    rep.contentType = "text/html; charset=utf-8";
    rep.extraHeaders["Cache-Control"] = "no-store";
    rep.extraHeaders["X-Frame-Options"] = "DENY";
    rep.body = kGuiPage;
    return true;
}

void StartWebGUI(HTTPServer& server) { server.RegisterHandler("/gui", true, HTTPReq_GUI); }

} // namespace bcp
