// Browser wallet GUI served by bcpd (GET /gui on the RPC port, -webgui).
// Parity: reference src/qt/ (bitcoin-qt: overview page with balances and recent transactions
// (overviewpage.cpp), send coins dialog with several recipients and coin control
// (sendcoinsdialog.cpp, coincontroldialog.cpp), receive coins with labels and payment requests
// (receivecoinsdialog.cpp, recentrequeststablemodel.cpp), address book with label editing
// (addressbookpage.cpp, editaddressdialog.cpp), transaction list with CSV export, wallet
// encryption, passphrase change, lock and backup (askpassphrasedialog.cpp, walletview.cpp
// backupWallet), transaction fee settings (sendcoinsdialog.cpp fee section), peers and banned
// peers with ban/unban (peertablemodel.cpp, bantablemodel.cpp, rpcconsole.cpp), network traffic
// totals (trafficgraphwidget.cpp), debug console with RPC history). Qt is not available here; the same functions are a single page that
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
<div id="morercp"></div><p><button onclick="addRcp()">Add recipient</button></p>
<label><input type="checkbox" id="sendsub"> subtract fee from amount</label>
<div>Comment</div><input class="wide" id="sendcomment">
<div id="passrow" style="display:none">Wallet passphrase <input type="password" id="sendpass"></div>
<p><button class="act" onclick="doSend()">Send</button> <span id="sendres"></span></p>
<details id="cc"><summary>Coin control</summary><p><button onclick="loadCoins()">List coins</button> Change address <input class="wide" id="ccchange"></p>
<table><thead><tr><th></th><th>Amount</th><th>Address</th><th>Conf.</th><th>Output</th></tr></thead><tbody id="cclist"></tbody></table></details></div>
<div class="card"><div>BIP70 payment request (hex or base64)</div><textarea class="wide" id="preq" rows="3"></textarea>
<p><button onclick="checkReq()">Check</button> <button class="act" onclick="payReq()">Pay request</button> <span id="preqres"></span></p>
<div id="preqinfo"></div></div></section>
<section id="receive"><div class="card">Label <input id="rcvlabel"> Amount <input id="rcvamt" type="number" step="0.00000001" min="0" style="width:130px">
Message <input id="rcvmsg"> <button class="act" onclick="newAddr()">Request payment</button>
<p class="mono" id="newaddr"></p></div>
<div class="card"><b>Requested payments</b> <button onclick="clearReqs()">Clear</button><table><thead><tr><th>Date</th><th>Label</th><th>Message</th><th>Amount</th><th>URI</th></tr></thead><tbody id="reqlist"></tbody></table></div>
<div class="card"><b>Receiving addresses</b><table><thead><tr><th>Address</th><th>Label</th><th>Received</th><th>Conf.</th></tr></thead><tbody id="rcvlist"></tbody></table></div></section>
<section id="transactions"><div class="card"><button onclick="exportCsv()">Export CSV</button></div><div class="card"><table><thead><tr><th>Date</th><th>Type</th><th>Address</th><th>Amount</th><th>Conf.</th><th>Txid</th></tr></thead><tbody id="txlist"></tbody></table></div></section>
<section id="addresses"><div class="card"><b>Receiving addresses</b> (label edits apply to the wallet's address book)<table><thead><tr><th>Address</th><th>Label</th><th></th></tr></thead><tbody id="ablist"></tbody></table></div>
<div class="card"><b>Address groupings</b> (addresses whose coins have been spent together)<table><thead><tr><th>Address</th><th>Balance</th><th>Label</th></tr></thead><tbody id="grplist"></tbody></table></div></section>
<section id="wallet"><div class="card"><b>Encryption</b> <span id="encstate"></span>
<div id="encnew">New passphrase <input type="password" id="encpass1"> Repeat <input type="password" id="encpass2"> <button class="act" onclick="encryptWallet()">Encrypt wallet</button></div>
<div id="encchg" style="display:none">Old passphrase <input type="password" id="chgold"> New <input type="password" id="chgnew1"> Repeat <input type="password" id="chgnew2"> <button class="act" onclick="changePass()">Change passphrase</button> <button onclick="lockWallet()">Lock now</button></div>
<p id="encres"></p></div>
<div class="card"><b>Backup</b> Destination on the node's host <input class="wide" id="bkpath" placeholder="/path/to/wallet-backup"> <button class="act" onclick="backupWallet()">Back up wallet</button> <span id="bkres"></span></div>
<div class="card"><b>Transaction fee</b><table><tbody id="feeinfo"></tbody></table>
Custom fee rate (BCP/kB, 0 = automatic) <input id="feerate" type="number" step="0.00000001" min="0" style="width:130px"> <button class="act" onclick="setFee()">Set</button> <span id="feeres"></span></div></section>
<section id="signverify"><div class="card"><b>Sign message</b><div>Address</div><input class="wide" id="smaddr">
<div>Message</div><textarea class="wide" id="smmsg" rows="3"></textarea>
<p><button class="act" onclick="signMsg()">Sign</button></p><p class="mono" id="smsig"></p></div>
<div class="card"><b>Verify message</b><div>Address</div><input class="wide" id="vmaddr">
<div>Message</div><textarea class="wide" id="vmmsg" rows="3"></textarea><div>Signature</div><input class="wide" id="vmsig">
<p><button class="act" onclick="verifyMsg()">Verify</button> <span id="vmres"></span></p></div></section>
<section id="peers"><div class="card"><table><tbody id="traffic"></tbody></table></div>
<div class="card"><table><thead><tr><th>Address</th><th>Client</th><th>Version</th><th>Direction</th><th>Height</th><th>Sent</th><th>Recv</th><th>Ping ms</th><th></th></tr></thead><tbody id="peerlist"></tbody></table></div>
<div class="card"><b>Banned peers</b> <button onclick="clearBans()">Unban all</button><table><thead><tr><th>Subnet</th><th>Banned until</th><th>Reason</th><th></th></tr></thead><tbody id="banlist"></tbody></table></div></section>
<section id="mining"><div class="card"><table><tbody id="mininfo"></tbody></table></div>
<div class="card"><table><tbody id="gpuinfo"></tbody></table></div>
<div class="card">Generate <input id="gencount" type="number" value="1" min="1" style="width:70px"> block(s) to this wallet (regtest)
<button class="act" onclick="doGenerate()">Generate</button> <span id="genres"></span></div></section>
<section id="console"><div class="card"><div id="conout"></div>
<input class="wide mono" id="conin" placeholder="method arg1 arg2 …  (e.g. getblockchaininfo, getblockhash 10; ↑/↓ history)"></div></section>
</main>
<script>
const TABS=[["overview","Overview"],["send","Send"],["receive","Receive"],["transactions","Transactions"],["addresses","Addresses"],["wallet","Wallet"],["signverify","Sign / verify"],["peers","Peers"],["mining","Mining"],["console","Console"]];
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
      const [b,u,w,n,tx,mp,up]=await Promise.all([rpc("getbalance"),rpc("getunconfirmedbalance"),rpc("getwalletinfo"),rpc("getnetworkinfo"),rpc("listtransactions",["*",10]),rpc("getmempoolinfo"),rpc("uptime")]);
      $("bal").textContent=amt(b);$("ubal").textContent=amt(u);$("ibal").textContent=amt(w.immature_balance);
      kv("chaininfo",Object.assign({},bc,{connections:n.connections,subversion:n.subversion,mempool_transactions:mp.size,mempool_bytes:mp.bytes,uptime_s:up}),["chain","blocks","headers","bestblockhash","difficulty","verificationprogress","connections","subversion","mempool_transactions","mempool_bytes","uptime_s"]);
      rows("recent",tx.reverse(),TXCOLS);}
    if(current=="receive"){rows("rcvlist",await rpc("listreceivedbyaddress",[0,true]),[[a=>a.address,'mono'],[a=>a.label||a.account],[a=>amt(a.amount)],[a=>a.confirmations]]);
      rows("reqlist",reqs().slice().reverse(),[[r=>date(r.time)],[r=>r.label],[r=>r.message],[r=>r.amount?amt(r.amount):""],[r=>r.uri,'mono']]);}
    if(current=="addresses"){
      const ab=await rpc("listreceivedbyaddress",[0,true]);
      $("ablist").innerHTML=ab.map((a,i)=>"<tr><td class='mono'>"+esc(a.address)+"</td><td><input id='lbl"+i+"' value='"+esc(a.label||a.account||"")+"'></td><td><button onclick=\"setLabel('"+esc(a.address)+"','lbl"+i+"')\">Save label</button></td></tr>").join("");
      rows("grplist",(await rpc("listaddressgroupings")).flat(),[[g=>g[0],'mono'],[g=>amt(g[1])],[g=>g[2]===undefined?"":g[2]]]);}
    if(current=="wallet"){
      const w=await rpc("getwalletinfo"),enc=w.unlocked_until!==undefined;
      $("encstate").textContent=enc?(w.unlocked_until>0?"encrypted, unlocked until "+date(w.unlocked_until):"encrypted, locked"):"not encrypted";
      $("encnew").style.display=enc?"none":"block";$("encchg").style.display=enc?"block":"none";
      const ef=await rpc("estimatesmartfee",[6]);
      kv("feeinfo",{paytxfee:w.paytxfee,estimated_rate_6_blocks:ef.feerate<0?"not enough data":ef.feerate,estimate_target_blocks:ef.blocks},["paytxfee","estimated_rate_6_blocks","estimate_target_blocks"]);}
    if(current=="transactions") rows("txlist",(await rpc("listtransactions",["*",200])).reverse(),TXCOLS.concat([[t=>t.txid,'mono']]));
    if(current=="peers"){
      const nt=await rpc("getnettotals");
      kv("traffic",{received_bytes:nt.totalbytesrecv,sent_bytes:nt.totalbytessent},["received_bytes","sent_bytes"]);
      const ps=await rpc("getpeerinfo");
      $("peerlist").innerHTML=ps.map(p=>"<tr>"+[[p.addr,'mono'],[p.subver],[p.version],[p.inbound?"in":"out"],[p.synced_blocks],[p.bytessent],[p.bytesrecv],[p.pingtime===undefined?"":Math.round(p.pingtime*1000)]].map(c=>"<td class='"+(c[1]||"")+"'>"+esc(c[0])+"</td>").join("")+
        "<td><button onclick=\"banPeer('"+esc(p.addr)+"')\">Ban 24 h</button></td></tr>").join("");
      $("banlist").innerHTML=(await rpc("listbanned")).map(b=>"<tr><td class='mono'>"+esc(b.address)+"</td><td>"+esc(date(b.banned_until))+"</td><td>"+esc(b.ban_reason||"")+
        "</td><td><button onclick=\"unban('"+esc(b.address)+"')\">Unban</button></td></tr>").join("");}
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
    const extra=[...document.querySelectorAll(".rcp")].map(r=>[r.querySelector(".rto").value.trim(),Number(r.querySelector(".ramt").value)]).filter(r=>r[0]);
    if(extra.length){const amts={};amts[to]=Number($("sendamt").value);for(const [a,v] of extra) amts[a]=(amts[a]||0)+v;
      const txid=await rpc("sendmany",["",amts,1,$("sendcomment").value,$("sendsub").checked?Object.keys(amts):[]]);
      $("sendres").innerHTML="<span class='ok'>sent "+esc(txid)+" to "+Object.keys(amts).length+" recipients</span>";$("sendpass").value="";return;}
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
  const q=v=>'"'+String(v==null?"":v).replace(/"/g,'""')+'"';
  const lines=[["Confirmed","Date","Type","Label","Address","Amount","ID"].map(q).join(",")].concat(txs.map(t=>
    [t.confirmations>0,new Date(t.time*1000).toISOString(),t.category,t.label||t.account||"",t.address||"",t.amount,t.txid].map(q).join(",")));
  const a=document.createElement("a");a.href=URL.createObjectURL(new Blob([lines.join("\n")],{type:"text/csv"}));
  a.download="transactions.csv";a.click();}
async function loadCoins(){const u=await rpc("listunspent",[0]);
  $("cclist").innerHTML=u.map(c=>"<tr><td><input type='checkbox' class='ccpick' data-txid='"+esc(c.txid)+"' data-vout='"+c.vout+"'></td><td>"+amt(c.amount)+
    "</td><td class='mono'>"+esc(c.address||"")+"</td><td>"+c.confirmations+"</td><td class='mono'>"+esc(c.txid.slice(0,16))+"…:"+c.vout+"</td></tr>").join("");}
function addRcp(){const d=document.createElement("div");d.className="rcp";
  d.innerHTML="Pay to <input class='wide rto' placeholder='address'> Amount (BCP) <input class='ramt' type='number' step='0.00000001' min='0'>";$("morercp").appendChild(d);}
// requested payments live in this browser (the reference keeps them in the wallet's destdata)
const reqs=()=>JSON.parse(localStorage.getItem("bcpRequests")||"[]");
function clearReqs(){localStorage.removeItem("bcpRequests");refresh("receive");}
async function newAddr(){try{const label=$("rcvlabel").value,msg=$("rcvmsg").value,v=Number($("rcvamt").value)||null;
  const a=await rpc("getnewaddress",[label]),uri=await rpc("formatbitcoinuri",[a,v,label,msg]);
  $("newaddr").textContent=uri;
  localStorage.setItem("bcpRequests",JSON.stringify(reqs().concat([{time:Math.floor(Date.now()/1000),label:label,message:msg,amount:v,uri:uri}])));refresh("receive");}
  catch(e){$("newaddr").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function setLabel(addr,id){try{await rpc("setaccount",[addr,$(id).value]);refresh("addresses");}catch(e){alert(e.message);}}
async function encryptWallet(){const a=$("encpass1").value;$("encres").textContent="";
  if(!a||a!=$("encpass2").value){$("encres").innerHTML="<span class='err'>the passphrases differ or are empty</span>";return;}
  try{const r=await rpc("encryptwallet",[a]);$("encres").innerHTML="<span class='ok'>"+esc(r)+"</span>";$("encpass1").value=$("encpass2").value="";refresh("wallet");}
  catch(e){$("encres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function changePass(){const n=$("chgnew1").value;$("encres").textContent="";
  if(!n||n!=$("chgnew2").value){$("encres").innerHTML="<span class='err'>the new passphrases differ or are empty</span>";return;}
  try{await rpc("walletpassphrasechange",[$("chgold").value,n]);$("encres").innerHTML="<span class='ok'>passphrase changed</span>";$("chgold").value=$("chgnew1").value=$("chgnew2").value="";}
  catch(e){$("encres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function lockWallet(){try{await rpc("walletlock");refresh("wallet");}catch(e){$("encres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function backupWallet(){try{await rpc("backupwallet",[$("bkpath").value.trim()]);$("bkres").innerHTML="<span class='ok'>backed up</span>";}
  catch(e){$("bkres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function setFee(){try{await rpc("settxfee",[Number($("feerate").value)]);$("feeres").innerHTML="<span class='ok'>set</span>";refresh("wallet");}
  catch(e){$("feeres").innerHTML="<span class='err'>"+esc(e.message)+"</span>";}}
async function banPeer(addr){try{await rpc("setban",[addr.replace(/:\d+$/,"").replace(/^\[|\]$/g,""),"add",86400]);refresh("peers");}catch(e){alert(e.message);}}
async function unban(sub){try{await rpc("setban",[sub,"remove"]);refresh("peers");}catch(e){alert(e.message);}}
async function clearBans(){try{await rpc("clearbanned");refresh("peers");}catch(e){alert(e.message);}}
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
