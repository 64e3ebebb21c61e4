// Wallet RPCs.
// Parity: reference src/wallet/rpcwallet.cpp:3332 command table (abandontransaction,
// addmultisigaddress, backupwallet, encryptwallet, getaccountaddress, getaccount,
// getaddressesbyaccount, getbalance, getnewaddress, getrawchangeaddress,
// getreceivedbyaccount, getreceivedbyaddress, gettransaction, getunconfirmedbalance,
// getwalletinfo, keypoolrefill, listaccounts, listaddressgroupings, listlockunspent,
// listreceivedbyaccount, listreceivedbyaddress, listsinceblock, listtransactions,
// listunspent, lockunspent, move, sendfrom, sendmany, sendtoaddress, setaccount,
// settxfee, signmessage, walletlock, walletpassphrasechange, walletpassphrase,
// fundrawtransaction, resendwallettransactions) and src/wallet/rpcdump.cpp
// (importprivkey, importaddress, importpubkey, importwallet, dumpprivkey, dumpwallet,
// importmulti, importprunedfunds, removeprunedfunds).
#include "consensus/merkleblock.h"
#include "node/node.h"
#include "node/policy.h"
#include "node/txmempool.h"
#include "node/validation.h"
#include "rpc/core_io.h"
#include "rpc/server.h"
#include "util/strencodings.h"
#include "wallet/bitcoinuri.h"
#include "wallet/paymentrequest.h"
#include "wallet/wallet.h"

#include <fstream>

namespace bcp {

static CWallet& Wallet(const JSONRPCRequest& req) {
    CWallet* w = nullptr;
    const std::string prefix = "/wallet/";
    if (req.URI.compare(0, prefix.size(), prefix) == 0) {
        const std::string name = req.URI.substr(prefix.size());
        for (CWallet* c : GetWallets())
            if (c->GetName() == name) w = c;
        if (!w) ThrowRPC(RPC_WALLET_ERROR, "Requested wallet does not exist or is not loaded");
    } else {
        w = GetWallet();
    }
    if (!w) ThrowRPC(RPC_METHOD_NOT_FOUND, "Method not found (disabled)");
    return *w;
}

static const CChainParams& P() { return Params(); }

static void EnsureWalletIsUnlocked(CWallet& w) {
    if (w.IsLocked())
        ThrowRPC(RPC_WALLET_UNLOCK_NEEDED, "Error: Please enter the wallet passphrase with walletpassphrase first.");
}

static std::string AccountFromValue(const UniValue& v) {
    const std::string a = v.get_str();
    if (a == "*") ThrowRPC(RPC_WALLET_INVALID_ACCOUNT_NAME, "Invalid account name");
    return a;
}

static CTxDestination ParseDest(const std::string& s) {
    const CTxDestination d = DecodeDestination(s, P());
    if (!d.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Bitcoin address");
    return d;
}

static void WalletTxToJSON(const CWalletTx& wtx, UniValue& entry) {
    const CBlockIndex* pi = nullptr;
    const int confirms = wtx.GetDepthInMainChain(&pi);
    entry.pushKV("confirmations", confirms);
    if (wtx.IsCoinBase()) entry.pushKV("generated", true);
    if (confirms > 0) {
        entry.pushKV("blockhash", wtx.hashBlock.GetHex());
        entry.pushKV("blockindex", wtx.nIndex);
        entry.pushKV("blocktime", pi ? pi->GetBlockTime() : (int64_t)0);
    } else {
        entry.pushKV("trusted", wtx.IsTrusted());
    }
    entry.pushKV("txid", wtx.GetHash().GetHex());
    UniValue conflicts(UniValue::VARR);
    for (const uint256& c : wtx.GetConflicts()) conflicts.push_back(c.GetHex());
    entry.pushKV("walletconflicts", conflicts);
    entry.pushKV("time", wtx.GetTxTime());
    entry.pushKV("timereceived", (int64_t)wtx.nTimeReceived);
    for (const auto& kv : wtx.mapValue) entry.pushKV(kv.first, kv.second);
}

static std::string LabelOf(CWallet& w, const CTxDestination& d) {
    auto it = w.mapAddressBook.find(d);
    return it == w.mapAddressBook.end() ? "" : it->second.name;
}

// ------------------------------------------------------------------ addresses
static UniValue getnewaddress(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() > 1) ThrowRPC(RPC_INVALID_PARAMS, "getnewaddress ( \"account\" )");
    std::string account;
    if (!req.params.empty() && !req.params[0].isNull()) account = AccountFromValue(req.params[0]);
    WalletLock l(w);
    if (!w.IsLocked()) w.TopUpKeyPool();
    CPubKey pub;
    if (!w.GetKeyFromPool(pub)) ThrowRPC(RPC_WALLET_KEYPOOL_RAN_OUT, "Error: Keypool ran out, please call keypoolrefill first");
    w.SetAddressBook(pub.GetID(), account, "receive");
    return EncodeDestination(pub.GetID(), P());
}

static UniValue getaccountaddress(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "getaccountaddress \"account\"");
    const std::string account = AccountFromValue(req.params[0]);
    CPubKey pub;
    if (!w.GetAccountPubkey(pub, account)) ThrowRPC(RPC_WALLET_KEYPOOL_RAN_OUT, "Error: Keypool ran out, please call keypoolrefill first");
    return EncodeDestination(pub.GetID(), P());
}

static UniValue getrawchangeaddress(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() > 1) ThrowRPC(RPC_INVALID_PARAMS, "getrawchangeaddress");
    WalletLock l(w);
    if (!w.IsLocked()) w.TopUpKeyPool();
    CReserveKey rk(&w);
    CPubKey pub;
    if (!rk.GetReservedKey(pub)) ThrowRPC(RPC_WALLET_KEYPOOL_RAN_OUT, "Error: Keypool ran out, please call keypoolrefill first");
    rk.KeepKey();
    return EncodeDestination(pub.GetID(), P());
}

static UniValue setaccount(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "setaccount \"address\" \"account\"");
    const CTxDestination d = ParseDest(req.params[0].get_str());
    std::string account;
    if (req.params.size() > 1) account = AccountFromValue(req.params[1]);
    WalletLock l(w);
    if (!IsMine(w, d)) ThrowRPC(RPC_MISC_ERROR, "setaccount can only be used with own address");
    w.SetAddressBook(d, account, "receive");
    return UniValue::NullUniValue;
}

static UniValue getaccount(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "getaccount \"address\"");
    const CTxDestination d = ParseDest(req.params[0].get_str());
    WalletLock l(w);
    return LabelOf(w, d);
}

static UniValue getaddressesbyaccount(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "getaddressesbyaccount \"account\"");
    const std::string account = AccountFromValue(req.params[0]);
    UniValue ret(UniValue::VARR);
    for (const CTxDestination& d : w.GetAccountAddresses(account)) ret.push_back(EncodeDestination(d, P()));
    return ret;
}

static UniValue addmultisigaddress(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 2 || req.params.size() > 3)
        ThrowRPC(RPC_INVALID_PARAMS, "addmultisigaddress nrequired [\"key\",...] ( \"account\" )");
    std::string account;
    if (req.params.size() > 2) account = AccountFromValue(req.params[2]);
    const int nRequired = req.params[0].get_int();
    const UniValue& keys = req.params[1].get_array();
    if (nRequired < 1) ThrowRPC(RPC_INVALID_PARAMETER, "a multisignature address must require at least one key to redeem");
    if ((int)keys.size() < nRequired)
        ThrowRPC(RPC_INVALID_PARAMETER, strprintf("not enough keys supplied (got %u keys, but need at least %d to redeem)",
                                                  (unsigned)keys.size(), nRequired));
    if (keys.size() > 16) ThrowRPC(RPC_INVALID_PARAMETER, "Number of addresses involved in the multisignature address creation > 16");
    std::vector<CPubKey> pubs;
    for (size_t i = 0; i < keys.size(); i++) {
        const std::string ks = keys[i].get_str();
        const CTxDestination d = DecodeDestination(ks, P());
        if (d.IsValid() && d.type == DestType::KEYID) {
            CPubKey pub;
            if (!w.GetPubKey(CKeyID(d.hash), pub))
                ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, strprintf("no full public key for address %s", ks.c_str()));
            pubs.push_back(pub);
        } else if (IsHex(ks)) {
            const std::vector<unsigned char> v = ParseHex(ks);
            CPubKey pub(v.begin(), v.end());
            if (!pub.IsFullyValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, " Invalid public key: " + ks);
            pubs.push_back(pub);
        } else {
            ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, " Invalid public key: " + ks);
        }
    }
    const CScript inner = GetScriptForMultisig(nRequired, pubs);
    if (inner.size() > MAX_SCRIPT_ELEMENT_SIZE)
        ThrowRPC(RPC_INVALID_PARAMETER, strprintf("redeemScript exceeds size limit: %u > %u", (unsigned)inner.size(),
                                                  (unsigned)MAX_SCRIPT_ELEMENT_SIZE));
    const CScriptID id(inner);
    w.AddCScript(inner);
    w.SetAddressBook(id, account, "send");
    return EncodeDestination(id, P());
}

// ------------------------------------------------------------------ sending
static void SendMoney(CWallet& w, const CTxDestination& address, Amount nValue, bool fSubtract, CWalletTx& wtxNew) {
    const Amount curBalance = w.GetBalance();
    if (nValue <= 0) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid amount");
    if (nValue > curBalance) ThrowRPC(RPC_WALLET_INSUFFICIENT_FUNDS, "Insufficient funds");
    if (w.fBroadcastTransactions && !GetNode()) ThrowRPC(RPC_CLIENT_P2P_DISABLED, "Error: Peer-to-peer functionality missing or disabled");
    CReserveKey rk(&w);
    Amount fee = 0;
    std::string err;
    int changePos = -1;
    std::vector<CRecipient> v{{GetScriptForDestination(address), nValue, fSubtract}};
    if (!w.CreateTransaction(v, wtxNew, rk, fee, changePos, err)) {
        if (!fSubtract && nValue + fee > curBalance)
            err = strprintf("Error: This transaction requires a transaction fee of at least %s", FormatMoney(fee).c_str());
        ThrowRPC(RPC_WALLET_ERROR, err);
    }
    CValidationState state;
    if (!w.CommitTransaction(wtxNew, rk, state))
        ThrowRPC(RPC_WALLET_ERROR, strprintf("Error: The transaction was rejected! Reason given: %s", state.GetRejectReason().c_str()));
}

static UniValue sendtoaddress(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 2 || req.params.size() > 5)
        ThrowRPC(RPC_INVALID_PARAMS, "sendtoaddress \"address\" amount ( \"comment\" \"comment_to\" subtractfeefromamount )");
    const CTxDestination d = ParseDest(req.params[0].get_str());
    const Amount nAmount = AmountFromValue(req.params[1]);
    if (nAmount <= 0) ThrowRPC(RPC_TYPE_ERROR, "Invalid amount for send");
    CWalletTx wtx;
    if (req.params.size() > 2 && !req.params[2].isNull() && !req.params[2].get_str().empty())
        wtx.mapValue["comment"] = req.params[2].get_str();
    if (req.params.size() > 3 && !req.params[3].isNull() && !req.params[3].get_str().empty())
        wtx.mapValue["to"] = req.params[3].get_str();
    bool fSubtract = false;
    if (req.params.size() > 4 && !req.params[4].isNull()) fSubtract = req.params[4].get_bool();
    EnsureWalletIsUnlocked(w);
    SendMoney(w, d, nAmount, fSubtract, wtx);
    return wtx.GetHash().GetHex();
}

static UniValue sendfrom(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 3 || req.params.size() > 6)
        ThrowRPC(RPC_INVALID_PARAMS, "sendfrom \"fromaccount\" \"toaddress\" amount ( minconf \"comment\" \"comment_to\" )");
    const std::string account = AccountFromValue(req.params[0]);
    const CTxDestination d = ParseDest(req.params[1].get_str());
    const Amount nAmount = AmountFromValue(req.params[2]);
    if (nAmount <= 0) ThrowRPC(RPC_TYPE_ERROR, "Invalid amount for send");
    int nMinDepth = 1;
    if (req.params.size() > 3) nMinDepth = req.params[3].get_int();
    CWalletTx wtx;
    wtx.strFromAccount = account;
    if (req.params.size() > 4 && !req.params[4].isNull() && !req.params[4].get_str().empty())
        wtx.mapValue["comment"] = req.params[4].get_str();
    if (req.params.size() > 5 && !req.params[5].isNull() && !req.params[5].get_str().empty())
        wtx.mapValue["to"] = req.params[5].get_str();
    EnsureWalletIsUnlocked(w);
    const Amount nBalance = w.GetAccountBalance(account, nMinDepth, ISMINE_SPENDABLE);
    if (nAmount > nBalance) ThrowRPC(RPC_WALLET_INSUFFICIENT_FUNDS, "Account has insufficient funds");
    SendMoney(w, d, nAmount, false, wtx);
    return wtx.GetHash().GetHex();
}

static UniValue sendmany(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 2 || req.params.size() > 5)
        ThrowRPC(RPC_INVALID_PARAMS, "sendmany \"fromaccount\" {\"address\":amount,...} ( minconf \"comment\" [\"address\",...] )");
    const std::string account = AccountFromValue(req.params[0]);
    const UniValue sendTo = req.params[1].get_obj();
    int nMinDepth = 1;
    if (req.params.size() > 2) nMinDepth = req.params[2].get_int();
    CWalletTx wtx;
    wtx.strFromAccount = account;
    if (req.params.size() > 3 && !req.params[3].isNull() && !req.params[3].get_str().empty())
        wtx.mapValue["comment"] = req.params[3].get_str();
    UniValue subtractFrom(UniValue::VARR);
    if (req.params.size() > 4 && !req.params[4].isNull()) subtractFrom = req.params[4].get_array();
    std::set<CTxDestination> seen;
    std::vector<CRecipient> vecSend;
    Amount totalAmount = 0;
    for (const std::string& name : sendTo.getKeys()) {
        const CTxDestination d = DecodeDestination(name, P());
        if (!d.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Bitcoin address: " + name);
        if (seen.count(d)) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, duplicated address: " + name);
        seen.insert(d);
        const Amount nAmount = AmountFromValue(sendTo[name]);
        if (nAmount <= 0) ThrowRPC(RPC_TYPE_ERROR, "Invalid amount for send");
        totalAmount += nAmount;
        bool fSub = false;
        for (size_t i = 0; i < subtractFrom.size(); i++)
            if (subtractFrom[i].get_str() == name) fSub = true;
        vecSend.push_back({GetScriptForDestination(d), nAmount, fSub});
    }
    EnsureWalletIsUnlocked(w);
    const Amount nBalance = w.GetAccountBalance(account, nMinDepth, ISMINE_SPENDABLE);
    if (totalAmount > nBalance) ThrowRPC(RPC_WALLET_INSUFFICIENT_FUNDS, "Account has insufficient funds");
    CReserveKey rk(&w);
    Amount fee = 0;
    int changePos = -1;
    std::string err;
    if (!w.CreateTransaction(vecSend, wtx, rk, fee, changePos, err)) ThrowRPC(RPC_WALLET_INSUFFICIENT_FUNDS, err);
    CValidationState state;
    if (!w.CommitTransaction(wtx, rk, state))
        ThrowRPC(RPC_WALLET_ERROR, "Transaction commit failed:: " + state.GetRejectReason());
    return wtx.GetHash().GetHex();
}

static UniValue fundrawtransaction(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "fundrawtransaction \"hexstring\" ( options )");
    CTxDestination changeAddress;
    int changePosition = -1;
    bool includeWatching = false, lockUnspents = false, reserveChangeKey = true, overrideFee = false;
    CFeeRate feeRate;
    std::set<int> subtractFrom;
    if (req.params.size() > 1 && !req.params[1].isNull()) {
        if (req.params[1].isBool()) {
            includeWatching = req.params[1].get_bool();
        } else {
            const UniValue& o = req.params[1].get_obj();
            // reference RPCTypeCheckObj(options, {...}, fAllowNull = true, fStrict = true)
            static const std::map<std::string, std::vector<UniValue::VType>> known = {
                {"changeAddress", {UniValue::VSTR}},   {"changePosition", {UniValue::VNUM}},
                {"includeWatching", {UniValue::VBOOL}}, {"lockUnspents", {UniValue::VBOOL}},
                {"reserveChangeKey", {UniValue::VBOOL}}, {"feeRate", {UniValue::VNUM, UniValue::VSTR}},
                {"subtractFeeFromOutputs", {UniValue::VARR}}};
            for (const std::string& k : o.getKeys()) {
                auto it = known.find(k);
                if (it == known.end()) ThrowRPC(RPC_TYPE_ERROR, strprintf("Unexpected key %s", k.c_str()));
                const UniValue& v = o[k];
                if (!v.isNull() && std::find(it->second.begin(), it->second.end(), v.getType()) == it->second.end())
                    ThrowRPC(RPC_TYPE_ERROR, strprintf("Expected type %s for %s, got %s", uvTypeName(it->second[0]),
                                                       k.c_str(), uvTypeName(v.getType())));
            }
            if (o.exists("changeAddress")) {
                changeAddress = DecodeDestination(o["changeAddress"].get_str(), P());
                if (!changeAddress.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "changeAddress must be a valid bitcoin address");
            }
            if (o.exists("changePosition")) changePosition = o["changePosition"].get_int();
            if (o.exists("includeWatching")) includeWatching = o["includeWatching"].get_bool();
            if (o.exists("lockUnspents")) lockUnspents = o["lockUnspents"].get_bool();
            if (o.exists("reserveChangeKey")) reserveChangeKey = o["reserveChangeKey"].get_bool();
            if (o.exists("feeRate")) {
                feeRate = CFeeRate(AmountFromValue(o["feeRate"]));
                overrideFee = true;
            }
            if (o.exists("subtractFeeFromOutputs")) {
                const UniValue& a = o["subtractFeeFromOutputs"].get_array();
                for (size_t i = 0; i < a.size(); i++) subtractFrom.insert(a[i].get_int());
            }
        }
    }
    CMutableTransaction tx;
    if (!DecodeHexTx(tx, req.params[0].get_str())) ThrowRPC(RPC_DESERIALIZATION_ERROR, "TX decode failed");
    if (tx.vout.empty()) ThrowRPC(RPC_INVALID_PARAMETER, "TX must have at least one output");
    if (changePosition != -1 && (changePosition < 0 || (size_t)changePosition > tx.vout.size()))
        ThrowRPC(RPC_INVALID_PARAMETER, "changePosition out of bounds");
    for (int pos : subtractFrom)
        if (pos < 0 || (size_t)pos >= tx.vout.size()) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, value out of range");
    Amount fee = 0;
    std::string err;
    if (!w.FundTransaction(tx, fee, overrideFee, feeRate, changePosition, err, includeWatching, lockUnspents,
                           subtractFrom, reserveChangeKey, changeAddress))
        ThrowRPC(RPC_WALLET_ERROR, err);
    UniValue r(UniValue::VOBJ);
    r.pushKV("hex", EncodeHexTx(CTransaction(tx)));
    r.pushKV("changepos", changePosition);
    r.pushKV("fee", ValueFromAmount(fee));
    return r;
}

// ------------------------------------------------------------------ balances / listing
static UniValue getbalance(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() > 3) ThrowRPC(RPC_INVALID_PARAMS, "getbalance ( \"account\" minconf include_watchonly )");
    std::lock_guard<CCriticalSection> lm(GetNode()->chainstate->cs());
    WalletLock l(w);
    if (req.params.empty()) return ValueFromAmount(w.GetBalance());
    int nMinDepth = 1;
    if (req.params.size() > 1 && !req.params[1].isNull()) nMinDepth = req.params[1].get_int();
    isminefilter filter = ISMINE_SPENDABLE;
    if (req.params.size() > 2 && !req.params[2].isNull() && req.params[2].get_bool()) filter = filter | ISMINE_WATCH_ONLY;
    if (req.params[0].get_str() == "*") {
        // all accounts: received - sent - fees over trusted, confirmed-enough txs
        Amount nBalance = 0;
        for (const auto& kv : w.mapWallet) {
            const CWalletTx& wtx = kv.second;
            if (!wtx.IsTrusted() || wtx.GetBlocksToMaturity() > 0) continue;
            std::list<COutputEntry> received, sent;
            Amount fee;
            std::string acc;
            wtx.GetAmounts(received, sent, fee, acc, filter);
            if (wtx.GetDepthInMainChain() >= nMinDepth)
                for (const COutputEntry& r : received) nBalance += r.amount;
            for (const COutputEntry& s : sent) nBalance -= s.amount;
            nBalance -= fee;
        }
        return ValueFromAmount(nBalance);
    }
    return ValueFromAmount(w.GetAccountBalance(AccountFromValue(req.params[0]), nMinDepth, filter));
}

static UniValue getunconfirmedbalance(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "getunconfirmedbalance");
    return ValueFromAmount(w.GetUnconfirmedBalance());
}

static Amount ReceivedByDests(CWallet& w, const std::set<CScript>& scripts, int nMinDepth) {
    Amount n = 0;
    WalletLock l(w);
    for (const auto& kv : w.mapWallet) {
        const CWalletTx& wtx = kv.second;
        if (wtx.IsCoinBase() || !IsFinalTx(*wtx.tx, GetNode()->chainstate->HeightNow() + 1, GetAdjustedTime())) continue;
        for (const CTxOut& o : wtx.tx->vout)
            if (scripts.count(o.scriptPubKey) && wtx.GetDepthInMainChain() >= nMinDepth) n += o.nValue;
    }
    return n;
}

static UniValue getreceivedbyaddress(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "getreceivedbyaddress \"address\" ( minconf )");
    const CTxDestination d = ParseDest(req.params[0].get_str());
    const CScript script = GetScriptForDestination(d);
    if (!IsMine(w, script)) return ValueFromAmount(0);
    int nMinDepth = 1;
    if (req.params.size() > 1) nMinDepth = req.params[1].get_int();
    return ValueFromAmount(ReceivedByDests(w, {script}, nMinDepth));
}

static UniValue getreceivedbyaccount(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "getreceivedbyaccount \"account\" ( minconf )");
    int nMinDepth = 1;
    if (req.params.size() > 1) nMinDepth = req.params[1].get_int();
    std::set<CScript> scripts;
    for (const CTxDestination& d : w.GetAccountAddresses(AccountFromValue(req.params[0])))
        if (IsMine(w, d)) scripts.insert(GetScriptForDestination(d));
    return ValueFromAmount(ReceivedByDests(w, scripts, nMinDepth));
}

static UniValue ListReceived(CWallet& w, const UniValue& params, bool fByAccounts) {
    int nMinDepth = 1;
    if (params.size() > 0 && !params[0].isNull()) nMinDepth = params[0].get_int();
    bool fIncludeEmpty = false;
    if (params.size() > 1 && !params[1].isNull()) fIncludeEmpty = params[1].get_bool();
    isminefilter filter = ISMINE_SPENDABLE;
    if (params.size() > 2 && !params[2].isNull() && params[2].get_bool()) filter = filter | ISMINE_WATCH_ONLY;
    struct Tally {
        Amount nAmount = 0;
        int nConf = INT32_MAX;
        std::vector<uint256> txids;
        bool fIsWatchonly = false;
    };
    WalletLock l(w);
    std::map<CTxDestination, Tally> mapTally;
    for (const auto& kv : w.mapWallet) {
        const CWalletTx& wtx = kv.second;
        if (wtx.IsCoinBase() || !IsFinalTx(*wtx.tx, GetNode()->chainstate->HeightNow() + 1, GetAdjustedTime())) continue;
        const int nDepth = wtx.GetDepthInMainChain();
        if (nDepth < nMinDepth) continue;
        for (const CTxOut& o : wtx.tx->vout) {
            CTxDestination d;
            if (!ExtractDestination(o.scriptPubKey, d)) continue;
            const isminefilter mine = IsMine(w, d);
            if (!(mine & filter)) continue;
            Tally& t = mapTally[d];
            t.nAmount += o.nValue;
            t.nConf = std::min(t.nConf, nDepth);
            t.txids.push_back(wtx.GetHash());
            if (mine & ISMINE_WATCH_ONLY) t.fIsWatchonly = true;
        }
    }
    UniValue ret(UniValue::VARR);
    std::map<std::string, Tally> mapAccountTally;
    for (const auto& kv : w.mapAddressBook) {
        const CTxDestination& d = kv.first;
        const std::string& account = kv.second.name;
        auto it = mapTally.find(d);
        if (it == mapTally.end() && !fIncludeEmpty) continue;
        Amount nAmount = 0;
        int nConf = INT32_MAX;
        bool fWatch = false;
        if (it != mapTally.end()) {
            nAmount = it->second.nAmount;
            nConf = it->second.nConf;
            fWatch = it->second.fIsWatchonly;
        }
        if (fByAccounts) {
            Tally& t = mapAccountTally[account];
            t.nAmount += nAmount;
            t.nConf = std::min(t.nConf, nConf);
            t.fIsWatchonly |= fWatch;
        } else {
            UniValue obj(UniValue::VOBJ);
            if (fWatch) obj.pushKV("involvesWatchonly", true);
            obj.pushKV("address", EncodeDestination(d, P()));
            obj.pushKV("account", account);
            obj.pushKV("amount", ValueFromAmount(nAmount));
            obj.pushKV("confirmations", nConf == INT32_MAX ? 0 : nConf);
            obj.pushKV("label", account);
            UniValue txids(UniValue::VARR);
            if (it != mapTally.end())
                for (const uint256& h : it->second.txids) txids.push_back(h.GetHex());
            obj.pushKV("txids", txids);
            ret.push_back(obj);
        }
    }
    if (fByAccounts) {
        for (const auto& kv : mapAccountTally) {
            UniValue obj(UniValue::VOBJ);
            if (kv.second.fIsWatchonly) obj.pushKV("involvesWatchonly", true);
            obj.pushKV("account", kv.first);
            obj.pushKV("amount", ValueFromAmount(kv.second.nAmount));
            obj.pushKV("confirmations", kv.second.nConf == INT32_MAX ? 0 : kv.second.nConf);
            obj.pushKV("label", kv.first);
            ret.push_back(obj);
        }
    }
    return ret;
}

static UniValue listreceivedbyaddress(const JSONRPCRequest& req) {
    if (req.params.size() > 3) ThrowRPC(RPC_INVALID_PARAMS, "listreceivedbyaddress ( minconf include_empty include_watchonly)");
    return ListReceived(Wallet(req), req.params, false);
}
static UniValue listreceivedbyaccount(const JSONRPCRequest& req) {
    if (req.params.size() > 3) ThrowRPC(RPC_INVALID_PARAMS, "listreceivedbyaccount ( minconf include_empty include_watchonly)");
    return ListReceived(Wallet(req), req.params, true);
}

static void ListTransactions(CWallet& w, const CWalletTx& wtx, const std::string& strAccount, int nMinDepth, bool fLong,
                             UniValue& ret, const isminefilter& filter) {
    Amount nFee;
    std::string strSentAccount;
    std::list<COutputEntry> listReceived, listSent;
    wtx.GetAmounts(listReceived, listSent, nFee, strSentAccount, filter);
    const bool fAllAccounts = strAccount == "*";
    const bool involvesWatchonly = wtx.IsFromMe(ISMINE_WATCH_ONLY);
    if ((!listSent.empty() || nFee != 0) && (fAllAccounts || strAccount == strSentAccount)) {
        for (const COutputEntry& s : listSent) {
            UniValue entry(UniValue::VOBJ);
            if (involvesWatchonly || (IsMine(w, s.destination) & ISMINE_WATCH_ONLY)) entry.pushKV("involvesWatchonly", true);
            entry.pushKV("account", strSentAccount);
            if (s.destination.IsValid()) entry.pushKV("address", EncodeDestination(s.destination, P()));
            entry.pushKV("category", "send");
            entry.pushKV("amount", ValueFromAmount(-s.amount));
            if (w.mapAddressBook.count(s.destination)) entry.pushKV("label", w.mapAddressBook[s.destination].name);
            entry.pushKV("vout", s.vout);
            entry.pushKV("fee", ValueFromAmount(-nFee));
            if (fLong) WalletTxToJSON(wtx, entry);
            entry.pushKV("abandoned", wtx.IsAbandoned());
            ret.push_back(entry);
        }
    }
    if (!listReceived.empty() && wtx.GetDepthInMainChain() >= nMinDepth) {
        for (const COutputEntry& r : listReceived) {
            std::string account;
            if (w.mapAddressBook.count(r.destination)) account = w.mapAddressBook[r.destination].name;
            if (!fAllAccounts && account != strAccount) continue;
            UniValue entry(UniValue::VOBJ);
            if (involvesWatchonly || (IsMine(w, r.destination) & ISMINE_WATCH_ONLY)) entry.pushKV("involvesWatchonly", true);
            entry.pushKV("account", account);
            if (r.destination.IsValid()) entry.pushKV("address", EncodeDestination(r.destination, P()));
            if (wtx.IsCoinBase()) {
                if (wtx.GetDepthInMainChain() < 1) entry.pushKV("category", "orphan");
                else if (wtx.GetBlocksToMaturity() > 0) entry.pushKV("category", "immature");
                else entry.pushKV("category", "generate");
            } else {
                entry.pushKV("category", "receive");
            }
            entry.pushKV("amount", ValueFromAmount(r.amount));
            if (w.mapAddressBook.count(r.destination)) entry.pushKV("label", account);
            entry.pushKV("vout", r.vout);
            if (fLong) WalletTxToJSON(wtx, entry);
            ret.push_back(entry);
        }
    }
}

static void AcentryToJSON(const CAccountingEntry& e, const std::string& strAccount, UniValue& ret) {
    if (strAccount != "*" && e.strAccount != strAccount) return;
    UniValue entry(UniValue::VOBJ);
    entry.pushKV("account", e.strAccount);
    entry.pushKV("category", "move");
    entry.pushKV("time", e.nTime);
    entry.pushKV("amount", ValueFromAmount(e.nCreditDebit));
    entry.pushKV("otheraccount", e.strOtherAccount);
    entry.pushKV("comment", e.strComment);
    ret.push_back(entry);
}

static UniValue listtransactions(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() > 4) ThrowRPC(RPC_INVALID_PARAMS, "listtransactions ( \"account\" count skip include_watchonly)");
    std::string strAccount = "*";
    if (!req.params.empty() && !req.params[0].isNull()) strAccount = req.params[0].get_str();
    int nCount = 10, nFrom = 0;
    if (req.params.size() > 1 && !req.params[1].isNull()) nCount = req.params[1].get_int();
    if (req.params.size() > 2 && !req.params[2].isNull()) nFrom = req.params[2].get_int();
    isminefilter filter = ISMINE_SPENDABLE;
    if (req.params.size() > 3 && !req.params[3].isNull() && req.params[3].get_bool()) filter = filter | ISMINE_WATCH_ONLY;
    if (nCount < 0) ThrowRPC(RPC_INVALID_PARAMETER, "Negative count");
    if (nFrom < 0) ThrowRPC(RPC_INVALID_PARAMETER, "Negative from");
    std::lock_guard<CCriticalSection> lm(GetNode()->chainstate->cs());
    WalletLock l(w);
    UniValue ret(UniValue::VARR);
    // newest first, then reverse the window (reference semantics)
    for (auto it = w.wtxOrdered.rbegin(); it != w.wtxOrdered.rend(); ++it) {
        if (it->second.first) ListTransactions(w, *it->second.first, strAccount, 0, true, ret, filter);
        if (it->second.second) AcentryToJSON(*it->second.second, strAccount, ret);
        if ((int)ret.size() >= nCount + nFrom) break;
    }
    if (nFrom > (int)ret.size()) nFrom = (int)ret.size();
    if (nFrom + nCount > (int)ret.size()) nCount = (int)ret.size() - nFrom;
    std::vector<UniValue> arr = ret.getValues();
    std::vector<UniValue> window(arr.begin() + nFrom, arr.begin() + nFrom + nCount);
    std::reverse(window.begin(), window.end());
    UniValue out(UniValue::VARR);
    for (const UniValue& v : window) out.push_back(v);
    return out;
}

static UniValue listaccounts(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "listaccounts ( minconf include_watchonly)");
    int nMinDepth = 1;
    if (!req.params.empty() && !req.params[0].isNull()) nMinDepth = req.params[0].get_int();
    isminefilter includeWatchonly = ISMINE_SPENDABLE;
    if (req.params.size() > 1 && !req.params[1].isNull() && req.params[1].get_bool())
        includeWatchonly = includeWatchonly | ISMINE_WATCH_ONLY;
    std::lock_guard<CCriticalSection> lm(GetNode()->chainstate->cs());
    WalletLock l(w);
    std::map<std::string, Amount> mapAccountBalances;
    for (const auto& kv : w.mapAddressBook)
        if (IsMine(w, kv.first) & includeWatchonly) mapAccountBalances[kv.second.name] = 0;
    for (const auto& kv : w.mapWallet) {
        const CWalletTx& wtx = kv.second;
        Amount nFee;
        std::string strSentAccount;
        std::list<COutputEntry> listReceived, listSent;
        const int nDepth = wtx.GetDepthInMainChain();
        if (wtx.GetBlocksToMaturity() > 0 || nDepth < 0) continue;
        wtx.GetAmounts(listReceived, listSent, nFee, strSentAccount, includeWatchonly);
        mapAccountBalances[strSentAccount] -= nFee;
        for (const COutputEntry& s : listSent) mapAccountBalances[strSentAccount] -= s.amount;
        if (nDepth >= nMinDepth)
            for (const COutputEntry& r : listReceived)
                mapAccountBalances[w.mapAddressBook.count(r.destination) ? w.mapAddressBook[r.destination].name : ""] += r.amount;
    }
    for (const CAccountingEntry& e : w.laccentries) mapAccountBalances[e.strAccount] += e.nCreditDebit;
    UniValue ret(UniValue::VOBJ);
    for (const auto& kv : mapAccountBalances) ret.pushKV(kv.first, ValueFromAmount(kv.second));
    return ret;
}

static UniValue listsinceblock(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() > 3) ThrowRPC(RPC_INVALID_PARAMS, "listsinceblock ( \"blockhash\" target_confirmations include_watchonly)");
    Chainstate& cs = *GetNode()->chainstate;
    std::lock_guard<CCriticalSection> lm(cs.cs());
    WalletLock l(w);
    const CBlockIndex* pindex = nullptr;
    int target_confirms = 1;
    isminefilter filter = ISMINE_SPENDABLE;
    if (!req.params.empty() && !req.params[0].isNull()) {
        // an unknown block lists everything; a block of a branch that is no longer active is
        // replaced by its fork point with the active chain, so transactions the reorg moved onto
        // the winning branch are reported (reference src/wallet/rpcwallet.cpp:2069-2082)
        uint256 h;
        h.SetHex(req.params[0].get_str());
        pindex = cs.LookupBlockIndex(h);
        if (pindex && cs.ActiveChain()[pindex->nHeight] != pindex) pindex = cs.ActiveChain().FindFork(pindex);
    }
    if (req.params.size() > 1 && !req.params[1].isNull()) {
        target_confirms = req.params[1].get_int();
        if (target_confirms < 1) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter");
    }
    if (req.params.size() > 2 && !req.params[2].isNull() && req.params[2].get_bool()) filter = filter | ISMINE_WATCH_ONLY;
    const int depth = pindex ? (1 + cs.Height() - pindex->nHeight) : -1;
    UniValue transactions(UniValue::VARR);
    for (const auto& kv : w.mapWallet)
        if (depth == -1 || kv.second.GetDepthInMainChain() < depth)
            ListTransactions(w, kv.second, "*", 0, true, transactions, filter);
    const CBlockIndex* pblockLast = cs.ActiveChain()[cs.Height() + 1 - target_confirms];
    const uint256 lastblock = pblockLast ? pblockLast->GetBlockHash() : uint256();
    UniValue ret(UniValue::VOBJ);
    ret.pushKV("transactions", transactions);
    ret.pushKV("lastblock", lastblock.GetHex());
    return ret;
}

static UniValue gettransaction(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "gettransaction \"txid\" ( include_watchonly )");
    const uint256 hash = ParseHashV(req.params[0], "txid");
    isminefilter filter = ISMINE_SPENDABLE;
    if (req.params.size() > 1 && !req.params[1].isNull() && req.params[1].get_bool()) filter = filter | ISMINE_WATCH_ONLY;
    std::lock_guard<CCriticalSection> lm(GetNode()->chainstate->cs());
    WalletLock l(w);
    auto it = w.mapWallet.find(hash);
    if (it == w.mapWallet.end()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid or non-wallet transaction id");
    const CWalletTx& wtx = it->second;
    const Amount nCredit = wtx.GetCredit(filter);
    const Amount nDebit = wtx.GetDebit(filter);
    const Amount nNet = nCredit - nDebit;
    const Amount nFee = wtx.IsFromMe(filter) ? wtx.tx->GetValueOut() - nDebit : 0;
    UniValue entry(UniValue::VOBJ);
    entry.pushKV("amount", ValueFromAmount(nNet - nFee));
    if (wtx.IsFromMe(filter)) entry.pushKV("fee", ValueFromAmount(nFee));
    WalletTxToJSON(wtx, entry);
    UniValue details(UniValue::VARR);
    ListTransactions(w, wtx, "*", 0, false, details, filter);
    entry.pushKV("details", details);
    entry.pushKV("hex", EncodeHexTx(*wtx.tx));
    return entry;
}

static UniValue abandontransaction(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "abandontransaction \"txid\"");
    const uint256 hash = ParseHashV(req.params[0], "txid");
    std::lock_guard<CCriticalSection> lm(GetNode()->chainstate->cs());
    WalletLock l(w);
    if (!w.mapWallet.count(hash)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid or non-wallet transaction id");
    if (!w.AbandonTransaction(hash)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Transaction not eligible for abandonment");
    return UniValue::NullUniValue;
}

static UniValue listunspent(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() > 4) ThrowRPC(RPC_INVALID_PARAMS, "listunspent ( minconf maxconf  [\"addresses\",...] [include_unsafe] )");
    int nMinDepth = 1, nMaxDepth = 9999999;
    if (!req.params.empty() && !req.params[0].isNull()) nMinDepth = req.params[0].get_int();
    if (req.params.size() > 1 && !req.params[1].isNull()) nMaxDepth = req.params[1].get_int();
    std::set<CTxDestination> dests;
    if (req.params.size() > 2 && !req.params[2].isNull()) {
        const UniValue& a = req.params[2].get_array();
        for (size_t i = 0; i < a.size(); i++) {
            const CTxDestination d = DecodeDestination(a[i].get_str(), P());
            if (!d.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Bitcoin address: " + a[i].get_str());
            if (!dests.insert(d).second) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, duplicated address: " + a[i].get_str());
        }
    }
    bool include_unsafe = true;
    if (req.params.size() > 3 && !req.params[3].isNull()) include_unsafe = req.params[3].get_bool();
    std::lock_guard<CCriticalSection> lm(GetNode()->chainstate->cs());
    WalletLock l(w);
    std::vector<COutput> vecOutputs;
    w.AvailableCoins(vecOutputs, !include_unsafe, nullptr, true);
    UniValue results(UniValue::VARR);
    for (const COutput& o : vecOutputs) {
        if (o.nDepth < nMinDepth || o.nDepth > nMaxDepth) continue;
        CTxDestination addr;
        const CScript& spk = o.tx->tx->vout[o.i].scriptPubKey;
        const bool fValid = ExtractDestination(spk, addr);
        if (!dests.empty() && (!fValid || !dests.count(addr))) continue;
        UniValue entry(UniValue::VOBJ);
        entry.pushKV("txid", o.tx->GetHash().GetHex());
        entry.pushKV("vout", o.i);
        if (fValid) {
            entry.pushKV("address", EncodeDestination(addr, P()));
            if (w.mapAddressBook.count(addr)) entry.pushKV("account", w.mapAddressBook[addr].name);
            if (addr.type == DestType::SCRIPTID) {
                CScript redeem;
                if (w.GetCScript(CScriptID(addr.hash), redeem)) entry.pushKV("redeemScript", HexStr(redeem.begin(), redeem.end()));
            }
        }
        entry.pushKV("scriptPubKey", HexStr(spk.begin(), spk.end()));
        entry.pushKV("amount", ValueFromAmount(o.tx->tx->vout[o.i].nValue));
        entry.pushKV("confirmations", o.nDepth);
        entry.pushKV("spendable", o.fSpendable);
        entry.pushKV("solvable", o.fSolvable);
        results.push_back(entry);
    }
    return results;
}

static UniValue lockunspent(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "lockunspent unlock ([{\"txid\":\"txid\",\"vout\":n},...])");
    const bool fUnlock = req.params[0].get_bool();
    if (req.params.size() == 1 || req.params[1].isNull()) {
        if (fUnlock) w.UnlockAllCoins();
        return true;
    }
    const UniValue& outputs = req.params[1].get_array();
    for (size_t i = 0; i < outputs.size(); i++) {
        const UniValue& o = outputs[i].get_obj();
        const std::string txid = find_value(o, "txid").get_str();
        if (!IsHex(txid)) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, expected hex txid");
        const int nOutput = find_value(o, "vout").get_int();
        if (nOutput < 0) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, vout must be positive");
        const COutPoint outpt(uint256S(txid), (uint32_t)nOutput);
        if (fUnlock) w.UnlockCoin(outpt);
        else w.LockCoin(outpt);
    }
    return true;
}

static UniValue listlockunspent(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "listlockunspent");
    UniValue ret(UniValue::VARR);
    for (const COutPoint& o : w.ListLockedCoins()) {
        UniValue obj(UniValue::VOBJ);
        obj.pushKV("txid", o.hash.GetHex());
        obj.pushKV("vout", (int)o.n);
        ret.push_back(obj);
    }
    return ret;
}

static UniValue listaddressgroupings(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "listaddressgroupings");
    std::lock_guard<CCriticalSection> lm(GetNode()->chainstate->cs());
    WalletLock l(w);
    UniValue jsonGroupings(UniValue::VARR);
    std::map<CTxDestination, Amount> balances = w.GetAddressBalances();
    for (const std::set<CTxDestination>& grouping : w.GetAddressGroupings()) {
        UniValue jsonGrouping(UniValue::VARR);
        for (const CTxDestination& address : grouping) {
            UniValue addressInfo(UniValue::VARR);
            addressInfo.push_back(EncodeDestination(address, P()));
            addressInfo.push_back(ValueFromAmount(balances[address]));
            if (w.mapAddressBook.count(address)) addressInfo.push_back(w.mapAddressBook[address].name);
            jsonGrouping.push_back(addressInfo);
        }
        jsonGroupings.push_back(jsonGrouping);
    }
    return jsonGroupings;
}

static UniValue move(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 3 || req.params.size() > 5)
        ThrowRPC(RPC_INVALID_PARAMS, "move \"fromaccount\" \"toaccount\" amount ( minconf \"comment\" )");
    const std::string from = AccountFromValue(req.params[0]);
    const std::string to = AccountFromValue(req.params[1]);
    const Amount nAmount = AmountFromValue(req.params[2]);
    if (nAmount <= 0) ThrowRPC(RPC_TYPE_ERROR, "Invalid amount for send");
    std::string comment;
    if (req.params.size() > 4) comment = req.params[4].get_str();
    WalletLock l(w);
    const int64_t nNow = GetAdjustedTime();
    CAccountingEntry debit;
    debit.nOrderPos = w.IncOrderPosNext();
    debit.strAccount = from;
    debit.nCreditDebit = -nAmount;
    debit.nTime = nNow;
    debit.strOtherAccount = to;
    debit.strComment = comment;
    w.AddAccountingEntry(debit);
    CAccountingEntry credit;
    credit.nOrderPos = w.IncOrderPosNext();
    credit.strAccount = to;
    credit.nCreditDebit = nAmount;
    credit.nTime = nNow;
    credit.strOtherAccount = from;
    credit.strComment = comment;
    w.AddAccountingEntry(credit);
    return true;
}

// ------------------------------------------------------------------ wallet state
static UniValue getwalletinfo(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "getwalletinfo");
    std::lock_guard<CCriticalSection> lm(GetNode()->chainstate->cs());
    WalletLock l(w);
    UniValue obj(UniValue::VOBJ);
    obj.pushKV("walletname", w.GetName());
    obj.pushKV("walletversion", w.GetVersion());
    obj.pushKV("balance", ValueFromAmount(w.GetBalance()));
    obj.pushKV("unconfirmed_balance", ValueFromAmount(w.GetUnconfirmedBalance()));
    obj.pushKV("immature_balance", ValueFromAmount(w.GetImmatureBalance()));
    obj.pushKV("txcount", (int64_t)w.mapWallet.size());
    obj.pushKV("keypoololdest", w.GetOldestKeyPoolTime());
    obj.pushKV("keypoolsize", (int64_t)w.KeypoolCountExternalKeys());
    if (w.IsCrypted()) obj.pushKV("unlocked_until", w.nRelockTime);
    obj.pushKV("paytxfee", ValueFromAmount(w.payTxFee.GetFeePerK()));
    if (w.IsHDEnabled()) obj.pushKV("hdmasterkeyid", w.GetHDChain().masterKeyID.GetHex());
    return obj;
}

static UniValue keypoolrefill(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() > 1) ThrowRPC(RPC_INVALID_PARAMS, "keypoolrefill ( newsize )");
    unsigned int kpSize = 0;
    if (!req.params.empty()) {
        if (req.params[0].get_int() < 0) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, expected valid size.");
        kpSize = (unsigned int)req.params[0].get_int();
    }
    EnsureWalletIsUnlocked(w);
    w.TopUpKeyPool(kpSize);
    if (w.KeypoolCountExternalKeys() < kpSize) ThrowRPC(RPC_WALLET_ERROR, "Error refreshing keypool.");
    return UniValue::NullUniValue;
}

static UniValue settxfee(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "settxfee amount");
    w.payTxFee = CFeeRate(AmountFromValue(req.params[0]));
    return true;
}

static UniValue backupwallet(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "backupwallet \"destination\"");
    if (!w.BackupWallet(req.params[0].get_str())) ThrowRPC(RPC_WALLET_ERROR, "Error: Wallet backup failed!");
    return UniValue::NullUniValue;
}

static void ScheduleRelock(CWallet& w, int64_t nSleepTime) {
    w.nRelockTime = GetTime() + nSleepTime;
    const int64_t when = w.nRelockTime;
    NodeContext* n = GetNode();
    if (n && n->scheduler)
        n->scheduler->ScheduleFromNow(
            [&w, when] {
                WalletLock l(w);
                if (w.nRelockTime == when) {
                    w.Lock();
                    w.nRelockTime = 0;
                }
            },
            nSleepTime * 1000);
}

static UniValue walletpassphrase(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (w.IsCrypted() && (req.params.size() != 2)) ThrowRPC(RPC_INVALID_PARAMS, "walletpassphrase \"passphrase\" timeout");
    if (!w.IsCrypted()) ThrowRPC(RPC_WALLET_WRONG_ENC_STATE, "Error: running with an unencrypted wallet, but walletpassphrase was called.");
    const std::string pass = req.params[0].get_str();
    if (pass.empty()) ThrowRPC(RPC_INVALID_PARAMS, "walletpassphrase <passphrase> <timeout>\nStores the wallet decryption key in memory for <timeout> seconds.");
    if (!w.Unlock(pass)) ThrowRPC(RPC_WALLET_PASSPHRASE_INCORRECT, "Error: The wallet passphrase entered was incorrect.");
    w.TopUpKeyPool();
    ScheduleRelock(w, req.params[1].get_int64());
    return UniValue::NullUniValue;
}

static UniValue walletpassphrasechange(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (w.IsCrypted() && req.params.size() != 2)
        ThrowRPC(RPC_INVALID_PARAMS, "walletpassphrasechange \"oldpassphrase\" \"newpassphrase\"");
    if (!w.IsCrypted())
        ThrowRPC(RPC_WALLET_WRONG_ENC_STATE, "Error: running with an unencrypted wallet, but walletpassphrasechange was called.");
    const std::string a = req.params[0].get_str(), b = req.params[1].get_str();
    if (a.empty() || b.empty()) ThrowRPC(RPC_INVALID_PARAMS, "walletpassphrasechange <oldpassphrase> <newpassphrase>");
    if (!w.ChangeWalletPassphrase(a, b)) ThrowRPC(RPC_WALLET_PASSPHRASE_INCORRECT, "Error: The wallet passphrase entered was incorrect.");
    return UniValue::NullUniValue;
}

static UniValue walletlock(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (w.IsCrypted() && !req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "walletlock");
    if (!w.IsCrypted()) ThrowRPC(RPC_WALLET_WRONG_ENC_STATE, "Error: running with an unencrypted wallet, but walletlock was called.");
    WalletLock l(w);
    w.Lock();
    w.nRelockTime = 0;
    return UniValue::NullUniValue;
}

static UniValue encryptwallet(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (!w.IsCrypted() && req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "encryptwallet \"passphrase\"");
    if (w.IsCrypted()) ThrowRPC(RPC_WALLET_WRONG_ENC_STATE, "Error: running with an encrypted wallet, but encryptwallet was called.");
    const std::string pass = req.params[0].get_str();
    if (pass.empty()) ThrowRPC(RPC_INVALID_PARAMS, "encryptwallet <passphrase>\nEncrypts the wallet with <passphrase>.");
    if (!w.EncryptWallet(pass)) ThrowRPC(RPC_WALLET_ENCRYPTION_FAILED, "Error: Failed to encrypt the wallet.");
    // the reference shuts the node down here to flush unencrypted key material from memory;
    // our store rewrote every key record, so the node keeps running
    return "wallet encrypted; The keypool has been flushed and a new HD seed was generated (if you are using HD). You "
           "need to make a new backup.";
}

static UniValue signmessage(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 2) ThrowRPC(RPC_INVALID_PARAMS, "signmessage \"address\" \"message\"");
    EnsureWalletIsUnlocked(w);
    const CTxDestination d = DecodeDestination(req.params[0].get_str(), P());
    if (!d.IsValid()) ThrowRPC(RPC_TYPE_ERROR, "Invalid address");
    if (d.type != DestType::KEYID) ThrowRPC(RPC_TYPE_ERROR, "Address does not refer to key");
    CKey key;
    if (!w.GetKey(CKeyID(d.hash), key)) ThrowRPC(RPC_WALLET_ERROR, "Private key not available");
    std::vector<unsigned char> sig;
    if (!key.SignCompact(MessageHash(req.params[1].get_str()), sig)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Sign failed");
    return EncodeBase64(sig.data(), sig.size());
}

static UniValue resendwallettransactions(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (!req.params.empty()) ThrowRPC(RPC_INVALID_PARAMS, "resendwallettransactions");
    if (!w.fBroadcastTransactions) ThrowRPC(RPC_WALLET_ERROR, "Error: Wallet transaction broadcasting is disabled with -walletbroadcast");
    UniValue ret(UniValue::VARR);
    for (const uint256& h : w.ResendWalletTransactionsBefore(GetTime())) ret.push_back(h.GetHex());
    return ret;
}

// ------------------------------------------------------------------ rpcdump
static void RescanFromGenesis(CWallet& w, int64_t nTimeBegin = 0) {
    Chainstate& cs = *GetNode()->chainstate;
    const CBlockIndex* start;
    {
        std::lock_guard<CCriticalSection> lm(cs.cs());
        start = cs.ActiveChain().Genesis();
        if (nTimeBegin > 0) {
            const CBlockIndex* t = cs.ActiveChain().FindEarliestAtLeast(nTimeBegin - 7200);
            if (t) start = t;
        }
    }
    w.ScanForWalletTransactions(start, true);
    w.ReacceptWalletTransactions();
}

// the single-key imports rescan from genesis, which a pruned node cannot (reference
// rpcdump.cpp:116-118, 234-236, 419-421, 461-463)
static bool PruneMode() { return GetNode()->chainstate->PruneMode(); }

static UniValue importprivkey(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 3) ThrowRPC(RPC_INVALID_PARAMS, "importprivkey \"bitcoinprivkey\" ( \"label\" ) ( rescan )");
    std::string label;
    if (req.params.size() > 1) label = req.params[1].get_str();
    bool fRescan = true;
    if (req.params.size() > 2) fRescan = req.params[2].get_bool();
    if (fRescan && PruneMode()) ThrowRPC(RPC_WALLET_ERROR, "Rescan is disabled in pruned mode");
    EnsureWalletIsUnlocked(w);
    const CKey key = DecodeSecret(req.params[0].get_str(), P());
    if (!key.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid private key encoding");
    const CPubKey pub = key.GetPubKey();
    const CKeyID vchAddress = pub.GetID();
    {
        WalletLock l(w);
        w.SetAddressBook(vchAddress, label, "receive");
        if (w.HaveKey(vchAddress)) return UniValue::NullUniValue;
        w.mapKeyMetadata[vchAddress].nCreateTime = 1;
        if (!w.AddKeyPubKey(key, pub)) ThrowRPC(RPC_WALLET_ERROR, "Error adding key to wallet");
        w.UpdateTimeFirstKey(1);
    }
    if (fRescan) RescanFromGenesis(w);
    return UniValue::NullUniValue;
}

static void ImportScript(CWallet& w, const CScript& script, const std::string& label, bool isRedeem) {
    if (!isRedeem && IsMine(w, script) == ISMINE_SPENDABLE)
        ThrowRPC(RPC_WALLET_ERROR, "The wallet already contains the private key for this address or script");
    if (isRedeem) {
        if (!w.HaveCScript(CScriptID(script)) && !w.AddCScript(script)) ThrowRPC(RPC_WALLET_ERROR, "Error adding p2sh redeemScript to wallet");
        ImportScript(w, GetScriptForDestination(CScriptID(script)), label, false);
    } else {
        CTxDestination d;
        if (ExtractDestination(script, d)) w.SetAddressBook(d, label, "receive");
        if (!w.HaveWatchOnly(script) && !w.AddWatchOnly(script, 0)) ThrowRPC(RPC_WALLET_ERROR, "Error adding address to wallet");
    }
}

static UniValue importaddress(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 4)
        ThrowRPC(RPC_INVALID_PARAMS, "importaddress \"address\" ( \"label\" rescan p2sh )");
    std::string label;
    if (req.params.size() > 1) label = req.params[1].get_str();
    bool fRescan = true;
    if (req.params.size() > 2) fRescan = req.params[2].get_bool();
    if (fRescan && PruneMode()) ThrowRPC(RPC_WALLET_ERROR, "Rescan is disabled in pruned mode");
    bool fP2SH = false;
    if (req.params.size() > 3) fP2SH = req.params[3].get_bool();
    const std::string s = req.params[0].get_str();
    const CTxDestination d = DecodeDestination(s, P());
    {
        WalletLock l(w);
        if (d.IsValid()) {
            if (fP2SH) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Cannot use the p2sh flag with an address - use a script instead");
            ImportScript(w, GetScriptForDestination(d), label, false);
        } else if (IsHex(s)) {
            const std::vector<unsigned char> data(ParseHex(s));
            ImportScript(w, CScript(data.begin(), data.end()), label, fP2SH);
        } else {
            ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Bitcoin address or script");
        }
    }
    if (fRescan) RescanFromGenesis(w);
    return UniValue::NullUniValue;
}

static UniValue importpubkey(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 3) ThrowRPC(RPC_INVALID_PARAMS, "importpubkey \"pubkey\" ( \"label\" rescan )");
    std::string label;
    if (req.params.size() > 1) label = req.params[1].get_str();
    bool fRescan = true;
    if (req.params.size() > 2) fRescan = req.params[2].get_bool();
    if (fRescan && PruneMode()) ThrowRPC(RPC_WALLET_ERROR, "Rescan is disabled in pruned mode");
    if (!IsHex(req.params[0].get_str())) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Pubkey must be a hex string");
    const std::vector<unsigned char> data(ParseHex(req.params[0].get_str()));
    const CPubKey pub(data.begin(), data.end());
    if (!pub.IsFullyValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Pubkey is not a valid public key");
    {
        WalletLock l(w);
        ImportScript(w, GetScriptForDestination(pub.GetID()), label, false);
        ImportScript(w, GetScriptForRawPubKey(pub), label, false);
    }
    if (fRescan) RescanFromGenesis(w);
    return UniValue::NullUniValue;
}

static UniValue dumpprivkey(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "dumpprivkey \"address\"");
    EnsureWalletIsUnlocked(w);
    const CTxDestination d = DecodeDestination(req.params[0].get_str(), P());
    if (!d.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Bitcoin address");
    if (d.type != DestType::KEYID) ThrowRPC(RPC_TYPE_ERROR, "Address does not refer to a key");
    CKey key;
    if (!w.GetKey(CKeyID(d.hash), key))
        ThrowRPC(RPC_WALLET_ERROR, "Private key for address " + req.params[0].get_str() + " is not known");
    return EncodeSecret(key, P());
}

static std::string EncodeDumpTime(int64_t t) {
    char buf[64];
    const time_t tt = (time_t)t;
    struct tm tmv;
    gmtime_r(&tt, &tmv);
    strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%SZ", &tmv);
    return buf;
}

static int64_t DecodeDumpTime(const std::string& s) {
    struct tm tmv = {};
    if (!strptime(s.c_str(), "%Y-%m-%dT%H:%M:%SZ", &tmv)) return 0;
    return (int64_t)timegm(&tmv);
}

static std::string EncodeDumpString(const std::string& s) {
    std::string r;
    for (unsigned char c : s) {
        if (c <= 32 || c >= 128 || c == '%') r += strprintf("%%%02x", c);
        else r += (char)c;
    }
    return r;
}

static std::string DecodeDumpString(const std::string& s) {
    std::string r;
    for (size_t i = 0; i < s.size(); i++) {
        if (s[i] == '%' && i + 2 < s.size() + 0 && i + 2 <= s.size() - 1 + 1) {
            r += (char)strtol(s.substr(i + 1, 2).c_str(), nullptr, 16);
            i += 2;
        } else {
            r += s[i];
        }
    }
    return r;
}

static UniValue dumpwallet(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "dumpwallet \"filename\"");
    EnsureWalletIsUnlocked(w);
    std::ofstream file(req.params[0].get_str());
    if (!file.is_open()) ThrowRPC(RPC_INVALID_PARAMETER, "Cannot open wallet dump file");
    Chainstate& cs = *GetNode()->chainstate;
    std::lock_guard<CCriticalSection> lm(cs.cs());
    WalletLock l(w);
    std::map<CKeyID, int64_t> mapKeyBirth;
    for (const CKeyID& id : w.GetKeys()) {
        auto it = w.mapKeyMetadata.find(id);
        mapKeyBirth[id] = it != w.mapKeyMetadata.end() ? it->second.nCreateTime : 0;
    }
    std::vector<std::pair<int64_t, CKeyID>> vKeyBirth;
    for (const auto& kv : mapKeyBirth) vKeyBirth.push_back({kv.second, kv.first});
    std::sort(vKeyBirth.begin(), vKeyBirth.end());
    file << strprintf("# Wallet dump created by Bitcoin Cash Plus %s\n", FormatFullVersion().c_str());
    file << strprintf("# * Created on %s\n", EncodeDumpTime(GetTime()).c_str());
    file << strprintf("# * Best block at time of backup was %i (%s),\n", cs.Height(), cs.Tip()->GetBlockHash().ToString().c_str());
    file << strprintf("#   mined on %s\n", EncodeDumpTime(cs.Tip()->GetBlockTime()).c_str());
    file << "\n";
    if (w.IsHDEnabled()) {
        CKey masterKey;
        if (w.GetKey(w.GetHDChain().masterKeyID, masterKey)) {
            CExtKey ext;
            ext.SetMaster(masterKey.begin(), masterKey.size());
            file << "# extended private masterkey: " << EncodeExtKey(ext, P()) << "\n\n";
        }
    }
    for (const auto& kb : vKeyBirth) {
        const CKeyID& keyid = kb.second;
        CKey key;
        if (!w.GetKey(keyid, key)) continue;
        const std::string strAddr = EncodeDestination(keyid, P());
        const std::string strTime = EncodeDumpTime(kb.first);
        const CKeyMetadata& meta = w.mapKeyMetadata[keyid];
        std::string tail;
        if (w.mapAddressBook.count(keyid)) {
            tail = strprintf("label=%s", EncodeDumpString(w.mapAddressBook[keyid].name).c_str());
        } else if (keyid == w.GetHDChain().masterKeyID) {
            tail = "hdmaster=1";
        } else {
            tail = "change=1";
        }
        file << strprintf("%s %s %s # addr=%s%s\n", EncodeSecret(key, P()).c_str(), strTime.c_str(), tail.c_str(),
                          strAddr.c_str(), meta.hdKeypath.empty() ? "" : (" hdkeypath=" + meta.hdKeypath).c_str());
    }
    file << "\n# End of dump\n";
    file.close();
    return UniValue::NullUniValue;
}

static UniValue importwallet(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "importwallet \"filename\"");
    if (PruneMode()) ThrowRPC(RPC_WALLET_ERROR, "Importing wallets is disabled in pruned mode");
    EnsureWalletIsUnlocked(w);
    std::ifstream file(req.params[0].get_str());
    if (!file.is_open()) ThrowRPC(RPC_INVALID_PARAMETER, "Cannot open wallet dump file");
    int64_t nTimeBegin = GetTime();
    bool fGood = true;
    std::string line;
    while (std::getline(file, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::vector<std::string> v;
        size_t pos = 0;
        while (pos < line.size()) {
            const size_t sp = line.find(' ', pos);
            v.push_back(line.substr(pos, sp == std::string::npos ? std::string::npos : sp - pos));
            if (sp == std::string::npos) break;
            pos = sp + 1;
        }
        if (v.size() < 2) continue;
        const CKey key = DecodeSecret(v[0], P());
        if (!key.IsValid()) continue;
        const CPubKey pub = key.GetPubKey();
        const CKeyID keyid = pub.GetID();
        WalletLock l(w);
        if (w.HaveKey(keyid)) continue;
        const int64_t nTime = DecodeDumpTime(v[1]);
        std::string label;
        bool fLabel = true;
        for (size_t k = 2; k < v.size(); k++) {
            if (v[k][0] == '#') break;
            if (v[k] == "change=1" || v[k] == "reserve=1") fLabel = false;
            if (v[k].compare(0, 6, "label=") == 0) {
                label = DecodeDumpString(v[k].substr(6));
                fLabel = true;
            }
        }
        w.mapKeyMetadata[keyid].nCreateTime = nTime;
        if (!w.AddKeyPubKey(key, pub)) {
            fGood = false;
            continue;
        }
        if (fLabel) w.SetAddressBook(keyid, label, "receive");
        nTimeBegin = std::min(nTimeBegin, nTime);
    }
    RescanFromGenesis(w, nTimeBegin);
    if (!fGood) ThrowRPC(RPC_WALLET_ERROR, "Error adding some keys to wallet");
    return UniValue::NullUniValue;
}

static UniValue importmulti(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "importmulti \"requests\" ( \"options\" )");
    const UniValue& requests = req.params[0].get_array();
    bool fRescan = true;
    if (req.params.size() > 1 && req.params[1].isObject() && req.params[1].exists("rescan"))
        fRescan = req.params[1]["rescan"].get_bool();
    UniValue response(UniValue::VARR);
    int64_t nLowestTimestamp = GetTime();
    bool anySuccess = false;
    for (size_t i = 0; i < requests.size(); i++) {
        const UniValue& d = requests[i];
        UniValue result(UniValue::VOBJ);
        // the timestamp is checked outside the per-request error capture: a missing or malformed
        // one fails the whole call (reference GetImportTimestamp, src/wallet/rpcdump.cpp:1065)
        int64_t ts = 0;
        if (!d.exists("timestamp")) ThrowRPC(RPC_TYPE_ERROR, "Missing required timestamp field for key");
        if (d["timestamp"].isNum()) ts = d["timestamp"].get_int64();
        else if (d["timestamp"].isStr() && d["timestamp"].get_str() == "now") ts = GetTime();
        else ThrowRPC(RPC_TYPE_ERROR, "Expected number or \"now\" timestamp value for key");
        try {
            // One request (reference src/wallet/rpcdump.cpp:692-1060 ProcessImport): the same
            // checks, error codes and messages, in the same order.
            const UniValue& spk = d["scriptPubKey"];
            if (!(spk.isObject() && spk.exists("address")) && !spk.isStr())
                ThrowRPC(RPC_INVALID_PARAMETER, "Invalid scriptPubKey");
            const std::string redeemHex = d.exists("redeemscript") ? d["redeemscript"].get_str() : "";
            const UniValue pubKeys = d.exists("pubkeys") ? d["pubkeys"].get_array() : UniValue(UniValue::VARR);
            const UniValue keys = d.exists("keys") ? d["keys"].get_array() : UniValue(UniValue::VARR);
            const bool internal = d.exists("internal") && d["internal"].get_bool();
            const bool watchOnly = d.exists("watchonly") && d["watchonly"].get_bool();
            const std::string label = d.exists("label") && !internal ? d["label"].get_str() : "";
            const bool isScript = spk.isStr();
            const bool isP2SH = !redeemHex.empty();
            CScript script;
            CTxDestination dest;
            if (!isScript) {
                dest = DecodeDestination(spk["address"].get_str(), P());
                if (!dest.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid address");
                script = GetScriptForDestination(dest);
            } else {
                if (!IsHex(spk.get_str())) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid scriptPubKey");
                const std::vector<unsigned char> data = ParseHex(spk.get_str());
                script = CScript(data.begin(), data.end());
            }
            if (watchOnly && keys.size()) ThrowRPC(RPC_INVALID_PARAMETER, "Incompatibility found between watchonly and keys");
            if (internal && d.exists("label")) ThrowRPC(RPC_INVALID_PARAMETER, "Incompatibility found between internal and label");
            if (!internal && isScript) ThrowRPC(RPC_INVALID_PARAMETER, "Internal must be set for hex scriptPubKey");
            if (!isP2SH && (keys.size() > 1 || pubKeys.size() > 1))
                ThrowRPC(RPC_INVALID_PARAMETER, "More than private key given for one address");
            if (isP2SH && !IsHex(redeemHex)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid redeem script");
            auto alreadyMine = [&](const CScript& s) {
                if (IsMine(w, s) == ISMINE_SPENDABLE)
                    ThrowRPC(RPC_WALLET_ERROR, "The wallet already contains the private key for this address or script");
            };
            auto watch = [&](const CScript& s) {
                if (!w.HaveWatchOnly(s) && !w.AddWatchOnly(s, ts)) ThrowRPC(RPC_WALLET_ERROR, "Error adding address to wallet");
            };
            auto decodeKey = [&](const UniValue& v) {
                const CKey key = DecodeSecret(v.get_str(), P());
                if (!key.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid private key encoding");
                return key;
            };
            // a key or pubkey must belong to the destination being imported
            auto consistent = [&](const CKeyID& id) {
                CTxDestination sd;
                if (!isScript ? !(dest == CTxDestination(id)) : (ExtractDestination(script, sd) && !(sd == CTxDestination(id))))
                    ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Consistency check failed");
            };
            bool success = false;
            WalletLock l(w);
            if (isP2SH) {
                const std::vector<unsigned char> rd = ParseHex(redeemHex);
                const CScript redeem(rd.begin(), rd.end());
                if (!script.IsPayToScriptHash()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid P2SH address / script");
                watch(redeem);
                if (!w.HaveCScript(CScriptID(redeem)) && !w.AddCScript(redeem))
                    ThrowRPC(RPC_WALLET_ERROR, "Error adding p2sh redeemScript to wallet");
                const CScript redeemDest = GetScriptForDestination(CTxDestination(CScriptID(redeem)));
                alreadyMine(redeemDest);
                watch(redeemDest);
                if (dest.IsValid()) w.SetAddressBook(dest, label, "receive");
                for (size_t k = 0; k < keys.size(); k++) {
                    const CKey key = decodeKey(keys[k]);
                    const CPubKey pub = key.GetPubKey();
                    w.SetAddressBook(pub.GetID(), label, "receive");
                    if (w.HaveKey(pub.GetID())) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Already have this key");
                    w.mapKeyMetadata[pub.GetID()].nCreateTime = ts;
                    if (!w.AddKeyPubKey(key, pub)) ThrowRPC(RPC_WALLET_ERROR, "Error adding key to wallet");
                    w.UpdateTimeFirstKey(ts);
                }
                success = true;
            } else {
                if (pubKeys.size() && keys.size() == 0) {
                    const std::string hex = pubKeys[0].get_str();
                    if (!IsHex(hex)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Pubkey must be a hex string");
                    const std::vector<unsigned char> pd = ParseHex(hex);
                    const CPubKey pub(pd.begin(), pd.end());
                    if (!pub.IsFullyValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Pubkey is not a valid public key");
                    consistent(pub.GetID());
                    const CScript pubKeyScript = GetScriptForDestination(CTxDestination(pub.GetID()));
                    alreadyMine(pubKeyScript);
                    watch(pubKeyScript);
                    w.SetAddressBook(pub.GetID(), label, "receive");
                    const CScript raw = GetScriptForRawPubKey(pub);
                    alreadyMine(raw);
                    watch(raw);
                    success = true;
                }
                if (keys.size()) {
                    const CKey key = decodeKey(keys[0]);
                    const CPubKey pub = key.GetPubKey();
                    consistent(pub.GetID());
                    w.SetAddressBook(pub.GetID(), label, "receive");
                    if (!w.HaveKey(pub.GetID())) {
                        w.mapKeyMetadata[pub.GetID()].nCreateTime = ts;
                        if (!w.AddKeyPubKey(key, pub)) ThrowRPC(RPC_WALLET_ERROR, "Error adding key to wallet");
                        w.UpdateTimeFirstKey(ts);
                        success = true;
                    }
                }
                if (pubKeys.size() == 0 && keys.size() == 0) {
                    alreadyMine(script);
                    watch(script);
                    if (!isScript && dest.IsValid()) w.SetAddressBook(dest, label, "receive");
                    success = true;
                }
            }
            if (!success) { // the key was already in the wallet (reference: "success": false, no error)
                result.pushKV("success", false);
                response.push_back(result);
                continue;
            }
            nLowestTimestamp = std::min(nLowestTimestamp, ts);
            anySuccess = true;
            result.pushKV("success", true);
        } catch (const JSONRPCException& e) {
            result.pushKV("success", false);
            result.pushKV("error", e.obj);
        } catch (const std::exception& e) {
            result.pushKV("success", false);
            result.pushKV("error", JSONRPCError(RPC_MISC_ERROR, e.what()));
        }
        response.push_back(result);
    }
    if (fRescan && anySuccess) RescanFromGenesis(w, nLowestTimestamp);
    return response;
}

static UniValue importprunedfunds(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 2) ThrowRPC(RPC_INVALID_PARAMS, "importprunedfunds \"rawtransaction\" \"txoutproof\"");
    CMutableTransaction mtx;
    if (!DecodeHexTx(mtx, req.params[0].get_str())) ThrowRPC(RPC_DESERIALIZATION_ERROR, "TX decode failed");
    const CTransactionRef tx = MakeTransactionRef(std::move(mtx));
    const std::vector<unsigned char> proof = ParseHex(req.params[1].get_str());
    CMerkleBlock mb;
    if (!DecodeTxOutProof(proof, mb)) ThrowRPC(RPC_DESERIALIZATION_ERROR, "Proof decode failed");
    std::vector<uint256> vMatch;
    std::vector<unsigned int> vIndex;
    Chainstate& cs = *GetNode()->chainstate;
    std::lock_guard<CCriticalSection> lm(cs.cs());
    if (mb.txn.ExtractMatches(vMatch, vIndex) != mb.header.hashMerkleRoot)
        ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Something wrong with merkleblock");
    const CBlockIndex* pi = cs.LookupBlockIndex(mb.header.GetHash());
    if (!pi || !cs.ActiveChain().Contains(pi)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Block not found in chain");
    int txnIndex = -1;
    for (size_t i = 0; i < vMatch.size(); i++)
        if (vMatch[i] == tx->GetHash()) txnIndex = (int)vIndex[i];
    if (txnIndex < 0) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Transaction given doesn't exist in proof");
    WalletLock l(w);
    if (!w.IsMine(*tx)) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "No addresses in wallet correspond to included transaction");
    CWalletTx wtx(&w, tx);
    wtx.hashBlock = pi->GetBlockHash();
    wtx.nIndex = txnIndex;
    w.AddToWallet(wtx, false);
    return UniValue::NullUniValue;
}

static UniValue removeprunedfunds(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "removeprunedfunds \"txid\"");
    const uint256 h = ParseHashV(req.params[0], "txid");
    WalletLock l(w);
    auto it = w.mapWallet.find(h);
    if (it == w.mapWallet.end()) ThrowRPC(RPC_INVALID_PARAMETER, "Transaction does not exist in wallet.");
    for (auto o = w.wtxOrdered.begin(); o != w.wtxOrdered.end();) {
        if (o->second.first == &it->second) o = w.wtxOrdered.erase(o);
        else ++o;
    }
    w.mapWallet.erase(it);
    w.DB().Erase(std::make_pair(std::string("tx"), h), true);
    return UniValue::NullUniValue;
}

// ---- BIP70 payment requests (reference src/qt/paymentserver.cpp processPaymentRequest :579-690,
// PaymentServer::fetchPaymentACK :692-760; the Qt dialog flow becomes two RPCs here).
static payments::PaymentRequestPlus ParsePaymentRequestParam(const UniValue& v, bool* sizeOk = nullptr) {
    const std::string in = v.get_str();
    std::vector<unsigned char> raw;
    if (IsHex(in)) {
        raw = ParseHex(in);
    } else {
        bool invalid = false;
        raw = DecodeBase64(in, &invalid);
        if (invalid) ThrowRPC(RPC_DESERIALIZATION_ERROR, "Payment request is neither hex nor base64");
    }
    if (sizeOk) *sizeOk = payments::VerifySize((int64_t)raw.size());
    else if (!payments::VerifySize((int64_t)raw.size()))
        ThrowRPC(RPC_INVALID_PARAMETER, strprintf("Payment request too large (%u bytes, allowed %d bytes)",
                                                  (unsigned)raw.size(), (int)payments::BIP70_MAX_PAYMENTREQUEST_SIZE));
    payments::PaymentRequestPlus pr;
    if (!pr.parse(std::string(raw.begin(), raw.end())))
        ThrowRPC(RPC_DESERIALIZATION_ERROR, "Payment request is not initialized (parse error)");
    return pr;
}

static payments::CertStore RootCertStore() {
    payments::CertStore cs;
    std::string err;
    if (!payments::LoadRootCertificates(gArgs.GetArg("-rootcertificates", "-system-"), cs, err))
        ThrowRPC(RPC_MISC_ERROR, err);
    cs.allow_self_signed_root = gArgs.GetBoolArg("-allowselfsignedrootcertificates", payments::DEFAULT_SELFSIGNED_ROOTCERTS);
    return cs;
}

static UniValue decodepaymentrequest(const JSONRPCRequest& req) {
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "decodepaymentrequest \"request\"");
    bool sizeOk = true;
    const payments::PaymentRequestPlus pr = ParsePaymentRequestParam(req.params[0], &sizeOk);
    const payments::PaymentDetails& d = pr.getDetails();
    UniValue r(UniValue::VOBJ);
    r.pushKV("payment_details_version", (int64_t)pr.getRequest().payment_details_version);
    r.pushKV("pki_type", pr.getRequest().pki_type);
    std::string merchant, merr;
    if (pr.getRequest().pki_type != "none") {
        if (!pr.getMerchant(RootCertStore(), merchant, &merr)) r.pushKV("merchant_error", merr);
    }
    r.pushKV("merchant", merchant);
    r.pushKV("network", d.network);
    r.pushKV("network_ok", payments::VerifyNetwork(d, P().NetworkIDString()));
    r.pushKV("time", (int64_t)d.time);
    if (d.has_expires) r.pushKV("expires", (int64_t)d.expires);
    r.pushKV("expired", payments::VerifyExpired(d, GetTime()));
    r.pushKV("size_ok", sizeOk);
    r.pushKV("memo", d.memo);
    r.pushKV("payment_url", d.payment_url);
    r.pushKV("merchant_data", HexStr(d.merchant_data.begin(), d.merchant_data.end()));
    UniValue outs(UniValue::VARR);
    Amount total = 0;
    bool amountsOk = true;
    for (const auto& [script, amount] : pr.getPayTo()) {
        UniValue o(UniValue::VOBJ);
        o.pushKV("amount", ValueFromAmount(amount));
        o.pushKV("amount_ok", payments::VerifyAmount(amount));
        amountsOk &= payments::VerifyAmount(amount);
        total += amount;
        CTxDestination dest;
        if (ExtractDestination(script, dest)) o.pushKV("address", EncodeDestination(dest, P()));
        o.pushKV("script", HexStr(script.begin(), script.end()));
        o.pushKV("dust", IsDust(CTxOut(amount, script), dustRelayFee));
        outs.push_back(o);
    }
    r.pushKV("outputs", outs);
    r.pushKV("total_ok", amountsOk && payments::VerifyAmount(total));
    return r;
}

static UniValue sendpaymentrequest(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 1 || req.params.size() > 2) ThrowRPC(RPC_INVALID_PARAMS, "sendpaymentrequest \"request\" ( \"memo\" )");
    const payments::PaymentRequestPlus pr = ParsePaymentRequestParam(req.params[0]);
    const payments::PaymentDetails& d = pr.getDetails();
    if (!payments::VerifyNetwork(d, P().NetworkIDString()))
        ThrowRPC(RPC_INVALID_PARAMETER, "Payment request rejected: network doesn't match client network");
    if (payments::VerifyExpired(d, GetTime())) ThrowRPC(RPC_INVALID_PARAMETER, "Payment request rejected: expired");
    std::string merchant;
    if (pr.getRequest().pki_type != "none") {
        std::string merr;
        if (!pr.getMerchant(RootCertStore(), merchant, &merr))
            ThrowRPC(RPC_INVALID_PARAMETER, "Payment request rejected: merchant authentication failed: " + merr);
    }
    std::vector<CRecipient> vecSend;
    Amount total = 0;
    for (const auto& [script, amount] : pr.getPayTo()) {
        if (!payments::VerifyAmount(amount)) ThrowRPC(RPC_INVALID_PARAMETER, "Payment request rejected: invalid amount");
        if (IsDust(CTxOut(amount, script), dustRelayFee))
            ThrowRPC(RPC_INVALID_PARAMETER, "Requested payment amount is too small (considered dust)");
        total += amount;
        if (!payments::VerifyAmount(total)) ThrowRPC(RPC_INVALID_PARAMETER, "Payment request rejected: invalid amount");
        vecSend.push_back({script, amount, false});
    }
    if (vecSend.empty()) ThrowRPC(RPC_INVALID_PARAMETER, "Payment request has no outputs");
    EnsureWalletIsUnlocked(w);
    CWalletTx wtx;
    if (!d.memo.empty()) wtx.mapValue["PaymentRequest"] = d.memo;
    if (!merchant.empty()) wtx.mapValue["to"] = merchant;
    CReserveKey rk(&w);
    Amount fee = 0;
    int changePos = -1;
    std::string err;
    if (!w.CreateTransaction(vecSend, wtx, rk, fee, changePos, err)) ThrowRPC(RPC_WALLET_INSUFFICIENT_FUNDS, err);
    CValidationState state;
    if (!w.CommitTransaction(wtx, rk, state))
        ThrowRPC(RPC_WALLET_ERROR, "Transaction commit failed:: " + state.GetRejectReason());
    // BIP70 Payment for the merchant's payment_url: merchant_data echoed, the signed
    // transaction, and a fresh refund address.
    payments::Payment pay;
    pay.has_merchant_data = d.has_merchant_data;
    pay.merchant_data = d.merchant_data;
    const std::string txhex = EncodeHexTx(*wtx.tx);
    const std::vector<unsigned char> txraw = ParseHex(txhex);
    pay.transactions.emplace_back(txraw.begin(), txraw.end());
    CPubKey refundKey;
    if (w.GetKeyFromPool(refundKey)) {
        const CScript s = GetScriptForDestination(CTxDestination(refundKey.GetID()));
        payments::Output o;
        o.has_script = true;
        o.script.assign(s.begin(), s.end());
        pay.refund_to.push_back(o);
    }
    if (req.params.size() > 1 && !req.params[1].isNull() && !req.params[1].get_str().empty()) {
        pay.has_memo = true;
        pay.memo = req.params[1].get_str();
    }
    const std::string payment = payments::SerializePayment(pay);
    UniValue r(UniValue::VOBJ);
    r.pushKV("txid", wtx.GetHash().GetHex());
    r.pushKV("merchant", merchant);
    r.pushKV("amount", ValueFromAmount(total));
    r.pushKV("fee", ValueFromAmount(fee));
    r.pushKV("payment_url", d.payment_url);
    r.pushKV("payment", HexStr(payment.begin(), payment.end()));
    r.pushKV("payment_mimetype", payments::BIP71_MIMETYPE_PAYMENT);
    return r;
}

// ---- BIP21 URIs (reference src/qt/guiutil.cpp parseBitcoinURI / formatBitcoinURI; the GUI's
// send and receive pages use these).
static UniValue parsebitcoinuri(const JSONRPCRequest& req) {
    if (req.params.size() != 1) ThrowRPC(RPC_INVALID_PARAMS, "parsebitcoinuri \"uri\"");
    SendCoinsRecipient r;
    const std::string uri = req.params[0].get_str();
    if (!ParseBitcoinURI(BitcoinURIScheme(true), uri, &r) && !ParseBitcoinURI(BitcoinURIScheme(false), uri, &r))
        ThrowRPC(RPC_INVALID_PARAMETER, "Invalid or unsupported payment URI");
    UniValue o(UniValue::VOBJ);
    o.pushKV("address", r.address);
    o.pushKV("isvalid", DecodeDestination(r.address, P()).IsValid());
    o.pushKV("amount", ValueFromAmount(r.amount));
    o.pushKV("label", r.label);
    o.pushKV("message", r.message);
    if (!r.paymentRequestUrl.empty()) o.pushKV("r", r.paymentRequestUrl);
    return o;
}

static UniValue formatbitcoinuri(const JSONRPCRequest& req) {
    if (req.params.size() < 1 || req.params.size() > 4)
        ThrowRPC(RPC_INVALID_PARAMS, "formatbitcoinuri \"address\" ( amount \"label\" \"message\" )");
    SendCoinsRecipient r;
    const CTxDestination d = ParseDest(req.params[0].get_str());
    r.address = EncodeDestination(d, P());
    if (req.params.size() > 1 && !req.params[1].isNull()) r.amount = AmountFromValue(req.params[1]);
    if (req.params.size() > 2 && !req.params[2].isNull()) r.label = req.params[2].get_str();
    if (req.params.size() > 3 && !req.params[3].isNull()) r.message = req.params[3].get_str();
    return FormatBitcoinURI(r, UseCashAddr());
}

// Coin control send (reference Qt SendCoinsDialog + CoinControlDialog: pay recipients from
// exactly the selected outputs, optional custom change address), used by the GUI send page.
static UniValue sendwithcoincontrol(const JSONRPCRequest& req) {
    CWallet& w = Wallet(req);
    if (req.params.size() < 2 || req.params.size() > 4)
        ThrowRPC(RPC_INVALID_PARAMS, "sendwithcoincontrol {\"address\":amount,...} [{\"txid\":\"id\",\"vout\":n},...] ( \"changeaddress\" [\"address\",...] )");
    const UniValue sendTo = req.params[0].get_obj();
    const UniValue inputs = req.params[1].get_array();
    CCoinControl cc;
    cc.fAllowOtherInputs = false;
    for (size_t i = 0; i < inputs.size(); i++) {
        const UniValue& o = inputs[i].get_obj();
        const int vout = find_value(o, "vout").get_int();
        if (vout < 0) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, vout must be positive");
        COutPoint op;
        op.hash = ParseHashO(o, "txid");
        op.n = (uint32_t)vout;
        cc.setSelected.insert(op);
    }
    if (cc.setSelected.empty()) ThrowRPC(RPC_INVALID_PARAMETER, "No inputs selected");
    if (req.params.size() > 2 && !req.params[2].isNull() && !req.params[2].get_str().empty()) {
        cc.destChange = DecodeDestination(req.params[2].get_str(), P());
        if (!cc.destChange.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid change address");
    }
    UniValue subtractFrom(UniValue::VARR);
    if (req.params.size() > 3 && !req.params[3].isNull()) subtractFrom = req.params[3].get_array();
    std::vector<CRecipient> vecSend;
    std::set<CTxDestination> seen;
    for (const std::string& name : sendTo.getKeys()) {
        const CTxDestination d = DecodeDestination(name, P());
        if (!d.IsValid()) ThrowRPC(RPC_INVALID_ADDRESS_OR_KEY, "Invalid Bitcoin address: " + name);
        if (!seen.insert(d).second) ThrowRPC(RPC_INVALID_PARAMETER, "Invalid parameter, duplicated address: " + name);
        const Amount nAmount = AmountFromValue(sendTo[name]);
        if (nAmount <= 0) ThrowRPC(RPC_TYPE_ERROR, "Invalid amount for send");
        bool fSub = false;
        for (size_t i = 0; i < subtractFrom.size(); i++)
            if (subtractFrom[i].get_str() == name) fSub = true;
        vecSend.push_back({GetScriptForDestination(d), nAmount, fSub});
    }
    if (vecSend.empty()) ThrowRPC(RPC_INVALID_PARAMETER, "No recipients");
    EnsureWalletIsUnlocked(w);
    CWalletTx wtx;
    CReserveKey rk(&w);
    Amount fee = 0;
    int changePos = -1;
    std::string err;
    if (!w.CreateTransaction(vecSend, wtx, rk, fee, changePos, err, &cc)) ThrowRPC(RPC_WALLET_INSUFFICIENT_FUNDS, err);
    CValidationState state;
    if (!w.CommitTransaction(wtx, rk, state))
        ThrowRPC(RPC_WALLET_ERROR, "Transaction commit failed:: " + state.GetRejectReason());
    UniValue r(UniValue::VOBJ);
    r.pushKV("txid", wtx.GetHash().GetHex());
    r.pushKV("fee", ValueFromAmount(fee));
    r.pushKV("changepos", changePos);
    return r;
}

void RegisterWalletRPCCommands(CRPCTable& t) {
    const CRPCCommand cmds[] = {
        {"rawtransactions", "fundrawtransaction", fundrawtransaction, false, {"hexstring", "options"}, "fundrawtransaction \"hexstring\" ( options )\nAdd inputs to a transaction until it has enough in value to meet its out value."},
        {"hidden", "resendwallettransactions", resendwallettransactions, true, {}, "resendwallettransactions\nImmediately re-broadcast unconfirmed wallet transactions to all peers."},
        {"wallet", "abandontransaction", abandontransaction, false, {"txid"}, "abandontransaction \"txid\"\nMark in-wallet transaction <txid> as abandoned."},
        {"wallet", "addmultisigaddress", addmultisigaddress, true, {"nrequired", "keys", "account"}, "addmultisigaddress nrequired [\"key\",...] ( \"account\" )\nAdd a nrequired-to-sign multisignature address to the wallet."},
        {"wallet", "backupwallet", backupwallet, true, {"destination"}, "backupwallet \"destination\"\nSafely copies current wallet file to destination."},
        {"wallet", "decodepaymentrequest", decodepaymentrequest, true, {"request"}, "decodepaymentrequest \"request\"\nDecode and check a BIP70 payment request (hex or base64): merchant authentication, network, expiry, amounts."},
        {"wallet", "sendpaymentrequest", sendpaymentrequest, false, {"request", "memo"}, "sendpaymentrequest \"request\" ( \"memo\" )\nPay a BIP70 payment request and return the BIP70 Payment message for its payment_url."},
        {"wallet", "parsebitcoinuri", parsebitcoinuri, true, {"uri"}, "parsebitcoinuri \"uri\"\nSplit a BIP21 payment URI into address, amount, label, message (and BIP72 r)."},
        {"wallet", "formatbitcoinuri", formatbitcoinuri, true, {"address", "amount", "label", "message"}, "formatbitcoinuri \"address\" ( amount \"label\" \"message\" )\nBuild a BIP21 payment URI."},
        {"wallet", "sendwithcoincontrol", sendwithcoincontrol, false, {"amounts", "inputs", "changeaddress", "subtractfeefrom"}, "sendwithcoincontrol {\"address\":amount,...} [{\"txid\":\"id\",\"vout\":n},...] ( \"changeaddress\" [\"address\",...] )\nSend to recipients spending only the selected outputs (coin control)."},
        {"wallet", "dumpprivkey", dumpprivkey, true, {"address"}, "dumpprivkey \"address\"\nReveals the private key corresponding to 'address'."},
        {"wallet", "dumpwallet", dumpwallet, true, {"filename"}, "dumpwallet \"filename\"\nDumps all wallet keys in a human-readable format."},
        {"wallet", "encryptwallet", encryptwallet, true, {"passphrase"}, "encryptwallet \"passphrase\"\nEncrypts the wallet with 'passphrase'."},
        {"wallet", "getaccountaddress", getaccountaddress, true, {"account"}, "getaccountaddress \"account\"\nDEPRECATED. Returns the current address for receiving payments to this account."},
        {"wallet", "getaccount", getaccount, true, {"address"}, "getaccount \"address\"\nDEPRECATED. Returns the account associated with the given address."},
        {"wallet", "getaddressesbyaccount", getaddressesbyaccount, true, {"account"}, "getaddressesbyaccount \"account\"\nDEPRECATED. Returns the list of addresses for the given account."},
        {"wallet", "getbalance", getbalance, false, {"account", "minconf", "include_watchonly"}, "getbalance ( \"account\" minconf include_watchonly )\nReturns the server's total available balance."},
        {"wallet", "getnewaddress", getnewaddress, true, {"account"}, "getnewaddress ( \"account\" )\nReturns a new address for receiving payments."},
        {"wallet", "getrawchangeaddress", getrawchangeaddress, true, {}, "getrawchangeaddress\nReturns a new address, for receiving change."},
        {"wallet", "getreceivedbyaccount", getreceivedbyaccount, false, {"account", "minconf"}, "getreceivedbyaccount \"account\" ( minconf )\nDEPRECATED. Returns the total amount received by addresses with <account>."},
        {"wallet", "getreceivedbyaddress", getreceivedbyaddress, false, {"address", "minconf"}, "getreceivedbyaddress \"address\" ( minconf )\nReturns the total amount received by the given address."},
        {"wallet", "gettransaction", gettransaction, false, {"txid", "include_watchonly"}, "gettransaction \"txid\" ( include_watchonly )\nGet detailed information about in-wallet transaction <txid>."},
        {"wallet", "getunconfirmedbalance", getunconfirmedbalance, false, {}, "getunconfirmedbalance\nReturns the server's total unconfirmed balance."},
        {"wallet", "getwalletinfo", getwalletinfo, false, {}, "getwalletinfo\nReturns an object containing various wallet state info."},
        {"wallet", "importmulti", importmulti, true, {"requests", "options"}, "importmulti \"requests\" ( \"options\" )\nImport addresses/scripts (with private or public keys, redeem script), rescanning all addresses in one-shot-only."},
        {"wallet", "importprivkey", importprivkey, true, {"privkey", "label", "rescan"}, "importprivkey \"privkey\" ( \"label\" ) ( rescan )\nAdds a private key to your wallet."},
        {"wallet", "importwallet", importwallet, true, {"filename"}, "importwallet \"filename\"\nImports keys from a wallet dump file."},
        {"wallet", "importaddress", importaddress, true, {"address", "label", "rescan", "p2sh"}, "importaddress \"address\" ( \"label\" rescan p2sh )\nAdds a script or address that can be watched as if it were in your wallet but cannot be used to spend."},
        {"wallet", "importprunedfunds", importprunedfunds, true, {"rawtransaction", "txoutproof"}, "importprunedfunds\nImports funds without rescan."},
        {"wallet", "importpubkey", importpubkey, true, {"pubkey", "label", "rescan"}, "importpubkey \"pubkey\" ( \"label\" rescan )\nAdds a public key (in hex) that can be watched as if it were in your wallet."},
        {"wallet", "keypoolrefill", keypoolrefill, true, {"newsize"}, "keypoolrefill ( newsize )\nFills the keypool."},
        {"wallet", "listaccounts", listaccounts, false, {"minconf", "include_watchonly"}, "listaccounts ( minconf include_watchonly)\nDEPRECATED. Returns Object that has account names as keys, account balances as values."},
        {"wallet", "listaddressgroupings", listaddressgroupings, false, {}, "listaddressgroupings\nLists groups of addresses which have had their common ownership made public."},
        {"wallet", "listlockunspent", listlockunspent, false, {}, "listlockunspent\nReturns list of temporarily unspendable outputs."},
        {"wallet", "listreceivedbyaccount", listreceivedbyaccount, false, {"minconf", "include_empty", "include_watchonly"}, "listreceivedbyaccount ( minconf include_empty include_watchonly)\nDEPRECATED. List balances by account."},
        {"wallet", "listreceivedbyaddress", listreceivedbyaddress, false, {"minconf", "include_empty", "include_watchonly"}, "listreceivedbyaddress ( minconf include_empty include_watchonly)\nList balances by receiving address."},
        {"wallet", "listsinceblock", listsinceblock, false, {"blockhash", "target_confirmations", "include_watchonly"}, "listsinceblock ( \"blockhash\" target_confirmations include_watchonly)\nGet all transactions in blocks since block [blockhash]."},
        {"wallet", "listtransactions", listtransactions, false, {"account", "count", "skip", "include_watchonly"}, "listtransactions ( \"account\" count skip include_watchonly)\nReturns up to 'count' most recent transactions."},
        {"wallet", "listunspent", listunspent, false, {"minconf", "maxconf", "addresses", "include_unsafe"}, "listunspent ( minconf maxconf  [\"addresses\",...] [include_unsafe] )\nReturns array of unspent transaction outputs."},
        {"wallet", "lockunspent", lockunspent, true, {"unlock", "transactions"}, "lockunspent unlock ([{\"txid\":\"txid\",\"vout\":n},...])\nUpdates list of temporarily unspendable outputs."},
        {"wallet", "move", move, false, {"fromaccount", "toaccount", "amount", "minconf", "comment"}, "move \"fromaccount\" \"toaccount\" amount ( minconf \"comment\" )\nDEPRECATED. Move a specified amount from one account in your wallet to another."},
        {"wallet", "removeprunedfunds", removeprunedfunds, true, {"txid"}, "removeprunedfunds \"txid\"\nDeletes the specified transaction from the wallet."},
        {"wallet", "sendfrom", sendfrom, false, {"fromaccount", "toaddress", "amount", "minconf", "comment", "comment_to"}, "sendfrom \"fromaccount\" \"toaddress\" amount ( minconf \"comment\" \"comment_to\" )\nDEPRECATED (use sendtoaddress). Sent an amount from an account to a bitcoin address."},
        {"wallet", "sendmany", sendmany, false, {"fromaccount", "amounts", "minconf", "comment", "subtractfeefrom"}, "sendmany \"fromaccount\" {\"address\":amount,...} ( minconf \"comment\" [\"address\",...] )\nSend multiple times."},
        {"wallet", "sendtoaddress", sendtoaddress, false, {"address", "amount", "comment", "comment_to", "subtractfeefromamount"}, "sendtoaddress \"address\" amount ( \"comment\" \"comment_to\" subtractfeefromamount )\nSend an amount to a given address."},
        {"wallet", "setaccount", setaccount, true, {"address", "account"}, "setaccount \"address\" \"account\"\nDEPRECATED. Sets the account associated with the given address."},
        {"wallet", "settxfee", settxfee, true, {"amount"}, "settxfee amount\nSet the transaction fee per kB. Overwrites the paytxfee parameter."},
        {"wallet", "signmessage", signmessage, true, {"address", "message"}, "signmessage \"address\" \"message\"\nSign a message with the private key of an address."},
        {"wallet", "walletlock", walletlock, true, {}, "walletlock\nRemoves the wallet encryption key from memory, locking the wallet."},
        {"wallet", "walletpassphrasechange", walletpassphrasechange, true, {"oldpassphrase", "newpassphrase"}, "walletpassphrasechange \"oldpassphrase\" \"newpassphrase\"\nChanges the wallet passphrase."},
        {"wallet", "walletpassphrase", walletpassphrase, true, {"passphrase", "timeout"}, "walletpassphrase \"passphrase\" timeout\nStores the wallet decryption key in memory for 'timeout' seconds."},
    };
    for (const auto& c : cmds) t.appendCommand(c.name, c);
}

} // namespace bcp
