// Wallet start/stop for bcpd (reference src/wallet/wallet.cpp CWallet::CreateWalletFromFile
// and InitLoadWallet: first-run HD seed + default key, keypool top-up, rescan from the
// stored best-block locator (or genesis with -rescan), -zapwallettxes, -walletbroadcast,
// -paytxfee/-txconfirmtarget; and the wallet hooks used by generate/getinfo/validateaddress).
#include "node/node.h"
#include "node/txmempool.h"
#include "node/ui_interface.h"
#include "node/validation.h"
#include "rpc/server.h"
#include "util/strencodings.h"
#include "wallet/bdbimport.h"
#include "wallet/wallet.h"

#include <cstdio>
#include <functional>
#include <sys/stat.h>

namespace bcp {

extern std::function<CScript()> g_walletMiningScript;
extern std::function<void(UniValue&)> g_walletGetInfo;
extern std::function<bool(const CTxDestination&, UniValue&)> g_walletDescribeAddress;

static std::vector<std::unique_ptr<CWallet>> g_ownedWallets;

std::string WalletHelp() {
    std::string s = "\nWallet options:\n";
    const std::pair<const char*, const char*> opts[] = {
        {"-disablewallet", "Do not load the wallet and disable wallet RPC calls"},
        {"-keypool=<n>", "Set key pool size to <n> (default: 100)"},
        {"-fallbackfee=<amt>", "A fee rate (in BCP/kB) used when fee estimation has insufficient data (default: 0.0002)"},
        {"-mintxfee=<amt>", "Fees (in BCP/kB) smaller than this are considered zero fee for transaction creation (default: 0.00001)"},
        {"-paytxfee=<amt>", "Fee (in BCP/kB) to add to transactions you send (default: 0.00)"},
        {"-rescan", "Rescan the block chain for missing wallet transactions on startup"},
        {"-salvagewallet", "Attempt to recover private keys from a corrupt wallet on startup"},
        {"-spendzeroconfchange", "Spend unconfirmed change when sending transactions (default: 1)"},
        {"-txconfirmtarget=<n>", "If paytxfee is not set, include enough fee so transactions begin confirmation within n blocks (default: 6)"},
        {"-usehd", "Use hierarchical deterministic key generation (HD) after BIP32. Only has effect during wallet creation/first start (default: 1)"},
        {"-wallet=<file>", "Specify wallet store (within data directory) (default: wallet.dat)"},
        {"-walletbroadcast", "Make the wallet broadcast transactions (default: 1)"},
        {"-rootcertificates=<file>", "Root certificates for BIP70 payment request merchant authentication, PEM or DER (default: -system-)"},
        {"-allowselfsignedrootcertificates", "Accept a self-signed merchant certificate in BIP70 payment requests (default: 0)"},
        {"-walletnotify=<cmd>", "Execute command when a wallet transaction changes (%s in cmd is replaced by TxID)"},
        {"-zapwallettxes", "Delete all wallet transactions and only recover those parts of the blockchain through -rescan on startup"},
        {"-upgradewallet", "Upgrade wallet to latest format on startup"},
    };
    for (const auto& o : opts) s += strprintf("  %-32s %s\n", o.first, o.second);
    if (gArgs.GetBoolArg("-help-debug", false)) {
        const std::pair<const char*, const char*> dbg[] = {
            {"-sendfreetransactions", "Send transactions as zero-fee transactions if possible (default: 0)"},
            {"-dblogsize=<n>", "Flush wallet database activity from memory to disk log every <n> megabytes (default: 100)"},
            {"-flushwallet", "Run a thread to flush wallet periodically (default: 1)"},
            {"-privdb", "Sets the DB_PRIVATE flag in the wallet db environment (default: 1; the wallet store is always private to this process)"},
            {"-walletrejectlongchains", "Wallet will not create transactions that violate mempool chain limits (default: 0)"},
        };
        s += "\nWallet debugging/testing options:\n";
        for (const auto& o : dbg) s += strprintf("  %-32s %s\n", o.first, o.second);
    }
    return s;
}

// -salvagewallet (reference CWalletDB::Recover): move the damaged store aside as
// <name>.<time>.bak, recover every intact batch from its log, and keep only the key records
// (private/encrypted keys, master keys, key metadata, HD chain); transactions come back
// through the rescan that -salvagewallet implies.
static bool SalvageWallet(const std::string& path, std::string& err) {
    struct stat st;
    if (stat(path.c_str(), &st) != 0) return true; // nothing to salvage
    const std::string bak = strprintf("%s.%lld.bak", path.c_str(), (long long)GetTime());
    if (rename(path.c_str(), bak.c_str()) != 0) {
        err = "Failed to rename " + path + " to " + bak;
        return false;
    }
    uint64_t skipped = 0;
    const std::map<std::string, std::string> recs = KVStore::Salvage(bak, &skipped);
    KVStore fresh(path, false, true);
    KVBatch b;
    size_t kept = 0;
    for (const auto& kv : recs) {
        std::string type;
        try {
            SpanReader r((const unsigned char*)kv.first.data(), kv.first.size(), SER_DISK, PROTOCOL_VERSION);
            r >> type;
        } catch (const std::exception&) {
            continue;
        }
        if (type == "key" || type == "wkey" || type == "mkey" || type == "ckey" || type == "keymeta" ||
            type == "hdchain") {
            b.WriteRaw(kv.first, kv.second);
            ++kept;
        }
    }
    if (!fresh.WriteBatch(b, true)) {
        err = "Salvage: writing the recovered wallet failed";
        return false;
    }
    LogPrintf("Salvage(aggressive) found %u records, kept %u key records, skipped %u damaged bytes\n",
              (unsigned)recs.size(), (unsigned)kept, (unsigned)skipped);
    return true;
}

static bool LoadOneWallet(NodeContext& node, const std::string& name, std::string& err) {
    Chainstate& cs = *node.chainstate;
    const std::string path = node.datadir + "/" + name;
    if (!BdbFileKind(path).empty()) {
        // a reference wallet.dat (Berkeley DB file or db_dump text): its records become this store
        size_t n = 0;
        if (!ImportBdbWalletFile(path, n, err)) {
            err = "Error importing Berkeley DB wallet " + name + ": " + err;
            return false;
        }
    }
    if (gArgs.GetBoolArg("-salvagewallet", false) && !SalvageWallet(path, err)) return false;
    std::unique_ptr<CWallet> w(new CWallet(name, path, false));
    bool firstRun = false;
    if (!w->Load(err, firstRun)) return false;
    if (gArgs.GetBoolArg("-zapwallettxes", false)) {
        KVBatch b;
        for (const auto& kv : w->mapWallet) b.Erase(std::make_pair(std::string("tx"), kv.first));
        w->DB().WriteBatch(b, true);
        w->mapWallet.clear();
        w->wtxOrdered.clear();
    }
    w->Attach(&cs, node.mempool.get());
    if (gArgs.IsArgSet("-paytxfee")) {
        int64_t n = 0;
        if (!ParseMoney(gArgs.GetArg("-paytxfee", ""), n)) {
            err = "Invalid amount for -paytxfee=<amount>: '" + gArgs.GetArg("-paytxfee", "") + "'";
            return false;
        }
        w->payTxFee = CFeeRate(n);
    }
    w->nTxConfirmTarget = (unsigned)gArgs.GetArg("-txconfirmtarget", (int64_t)DEFAULT_TX_CONFIRM_TARGET);
    w->fBroadcastTransactions = gArgs.GetBoolArg("-walletbroadcast", DEFAULT_WALLETBROADCAST);
    w->fSendFreeTransactions = gArgs.GetBoolArg("-sendfreetransactions", DEFAULT_SEND_FREE_TRANSACTIONS);
    // -upgradewallet[=<max version>], implied on first run (reference wallet.cpp:4063-4081)
    if (gArgs.GetBoolArg("-upgradewallet", firstRun)) {
        int64_t nMaxVersion = gArgs.GetArg("-upgradewallet", (int64_t)0);
        if (nMaxVersion == 0 || nMaxVersion == 1) { // no argument (a bare flag reads as 1)
            LogPrintf("Performing wallet upgrade to %i\n", WALLET_FEATURE_LATEST);
            nMaxVersion = CLIENT_VERSION;
            w->SetMinVersion(WALLET_FEATURE_LATEST);
        } else {
            LogPrintf("Allowing wallet upgrade up to %i\n", (int)nMaxVersion);
        }
        if (nMaxVersion < w->GetVersion()) {
            err = "Cannot downgrade wallet";
            return false;
        }
        w->nWalletMaxVersion = (int)nMaxVersion;
    }
    if (firstRun) {
        if (gArgs.GetBoolArg("-usehd", true) && !w->IsHDEnabled()) {
            if (!w->SetHDMasterKey(w->GenerateNewHDMasterKey())) {
                err = "Storing master key failed";
                return false;
            }
            w->SetMinVersion(WALLET_FEATURE_HD); // only HD-aware clients may open it
        }
        w->TopUpKeyPool();
        CPubKey def;
        if (w->GetKeyFromPool(def)) {
            w->vchDefaultKey = def;
            w->SetAddressBook(def.GetID(), "", "receive");
            w->DB().Write(std::string("defaultkey"), def, true);
        }
    }
    // rescan from the wallet's best block (or genesis) to the tip
    const CBlockIndex* start = nullptr;
    {
        std::lock_guard<CCriticalSection> l(cs.cs());
        CBlockLocator loc;
        if (!gArgs.GetBoolArg("-rescan", false) && !gArgs.GetBoolArg("-zapwallettxes", false) &&
            !gArgs.GetBoolArg("-salvagewallet", false) &&
            w->DB().Read(std::string("bestblock"), loc)) {
            start = cs.FindForkInGlobalIndex(loc);
        } else {
            start = cs.ActiveChain().Genesis();
        }
        if (start && start != cs.Tip()) start = cs.ActiveChain().Next(start) ? start : nullptr;
    }
    GetMainSignals().Register(w.get());
    uiInterface.LoadWallet(w.get());
    if (start && start != cs.TipNow()) {
        LogPrintf("Rescanning last %i blocks (from block %i)...\n", cs.HeightNow() - start->nHeight, start->nHeight);
        w->ScanForWalletTransactions(start, true);
        std::lock_guard<CCriticalSection> l(cs.cs());
        w->SetBestChain(cs.ActiveChain().GetLocator());
    }
    w->ReacceptWalletTransactions();
    g_ownedWallets.push_back(std::move(w));
    return true;
}

bool StartWallet(NodeContext& node, std::string& err) {
    if (gArgs.GetBoolArg("-disablewallet", false)) {
        LogPrintf("Wallet disabled!\n");
        return true;
    }
    // wallet parameter interaction (reference wallet.cpp:4268-4368 ParameterInteraction / InitAutoStart)
    if (gArgs.GetBoolArg("-sysperms", false)) {
        err = "-sysperms is not allowed in combination with enabled wallet functionality";
        return false;
    }
    if (gArgs.GetBoolArg("-sendfreetransactions", DEFAULT_SEND_FREE_TRANSACTIONS) &&
        gArgs.GetArg("-limitfreerelay", (int64_t)0) <= 0) {
        err = "Creation of free transactions with their relay disabled is not supported.";
        return false;
    }
    std::vector<std::string> names = gArgs.GetArgs("-wallet");
    if (names.empty()) names.push_back("wallet.dat");
    for (const std::string& n : names) {
        if (n.find('/') != std::string::npos) {
            err = "Wallet parameter must only specify a filename (not a path): " + n;
            return false;
        }
        if (!LoadOneWallet(node, n, err)) return false;
    }
    CWallet* w = g_ownedWallets.front().get();
    node.wallet = w;
    node.keystore = w;
    g_walletMiningScript = [w]() {
        CReserveKey rk(w);
        CPubKey pub;
        if (!rk.GetReservedKey(pub)) ThrowRPC(RPC_WALLET_KEYPOOL_RAN_OUT, "Error: Keypool ran out, please call keypoolrefill first");
        rk.KeepKey();
        // pay-to-pubkey, as the reference's CWallet::GetScriptForMining (src/wallet/wallet.cpp:3711)
        return GetScriptForRawPubKey(pub);
    };
    g_walletGetInfo = [w](UniValue& obj) {
        obj.pushKV("walletversion", w->GetVersion());
        obj.pushKV("balance", ValueFromAmount(w->GetBalance()));
        obj.pushKV("keypoololdest", w->GetOldestKeyPoolTime());
        obj.pushKV("keypoolsize", (int64_t)w->KeypoolCountExternalKeys());
        if (w->IsCrypted()) obj.pushKV("unlocked_until", w->nRelockTime);
        obj.pushKV("paytxfee", ValueFromAmount(w->payTxFee.GetFeePerK()));
    };
    g_walletDescribeAddress = [w](const CTxDestination& d, UniValue& ret) {
        WalletLock l(*w);
        const isminetype mine = IsMine(*w, d);
        ret.pushKV("ismine", (mine & ISMINE_SPENDABLE) != 0);
        ret.pushKV("iswatchonly", (mine & ISMINE_WATCH_ONLY) != 0);
        if (d.type == DestType::KEYID) {
            CPubKey pub;
            ret.pushKV("isscript", false);
            if (w->GetPubKey(CKeyID(d.hash), pub)) {
                ret.pushKV("pubkey", HexStr(pub.begin(), pub.end()));
                ret.pushKV("iscompressed", pub.IsCompressed());
            }
        } else if (d.type == DestType::SCRIPTID) {
            ret.pushKV("isscript", true);
            CScript s;
            if (w->GetCScript(CScriptID(d.hash), s)) ret.pushKV("hex", HexStr(s.begin(), s.end()));
        }
        auto it = w->mapAddressBook.find(d);
        if (it != w->mapAddressBook.end()) ret.pushKV("account", it->second.name);
        if (d.type == DestType::KEYID) {
            auto m = w->mapKeyMetadata.find(CKeyID(d.hash));
            if (m != w->mapKeyMetadata.end()) {
                ret.pushKV("timestamp", m->second.nCreateTime);
                if (!m->second.hdKeypath.empty()) {
                    ret.pushKV("hdkeypath", m->second.hdKeypath);
                    ret.pushKV("hdmasterkeyid", m->second.hdMasterKeyID.GetHex());
                }
            }
        }
        return true;
    };
    // -flushwallet: make the wallet stores durable every few seconds (reference walletdb.cpp:750
    // ThreadFlushWalletDB; the stores here are write-ahead logged, so this is an fsync point)
    if (node.scheduler && gArgs.GetBoolArg("-flushwallet", DEFAULT_FLUSHWALLET))
        node.scheduler->ScheduleEvery(
            [] {
                for (CWallet* x : GetWallets()) x->FlushIfDirty();
            },
            2 * 1000);
    // periodic rebroadcast of unconfirmed wallet transactions
    if (node.scheduler)
        node.scheduler->ScheduleEvery(
            [] {
                for (CWallet* x : GetWallets()) x->ResendWalletTransactions(GetTime());
            },
            60 * 1000);
    return true;
}

void StopWallet(NodeContext& node) {
    g_walletMiningScript = nullptr;
    g_walletGetInfo = nullptr;
    g_walletDescribeAddress = nullptr;
    for (auto& w : g_ownedWallets) {
        GetMainSignals().Unregister(w.get());
        w->Flush();
    }
    node.wallet = nullptr;
    node.keystore = nullptr;
    g_ownedWallets.clear();
}

} // namespace bcp
