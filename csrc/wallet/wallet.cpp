#include "wallet/wallet.h"

#include <filesystem>
#include "node/ui_interface.h"
#include "consensus/params.h"
#include "consensus/tx_verify.h"
#include "node/policy.h"
#include "node/txmempool.h"
#include "node/validation.h"
#include "script/sign.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <algorithm>
#include <limits>
#include <functional>
#include <random>

namespace bcp {

extern std::function<void(const uint256&)> g_relayTransaction;

static const unsigned int BIP32_HARDENED_KEY_LIMIT = 0x80000000;

const uint256 CWalletTx::ABANDON_HASH = uint256S("0000000000000000000000000000000000000000000000000000000000000001");

static std::vector<CWallet*> g_wallets;
static std::mutex cs_wallets;
CWallet* GetWallet() {
    std::lock_guard<std::mutex> l(cs_wallets);
    return g_wallets.empty() ? nullptr : g_wallets.front();
}
std::vector<CWallet*> GetWallets() {
    std::lock_guard<std::mutex> l(cs_wallets);
    return g_wallets;
}

// ------------------------------------------------------------------ record keys
namespace {
struct DestKey {
    CTxDestination d;
    template <typename S> void Serialize(S& s) const {
        const uint8_t t = (uint8_t)d.type;
        ::bcp::Serialize(s, t);
        ::bcp::Serialize(s, d.hash);
    }
    template <typename S> void Unserialize(S& s) {
        uint8_t t;
        ::bcp::Unserialize(s, t);
        d.type = (DestType)t;
        ::bcp::Unserialize(s, d.hash);
    }
};
template <typename T> std::pair<std::string, T> K(const char* type, const T& v) { return {std::string(type), v}; }
} // namespace

// ------------------------------------------------------------------ IsMine
isminetype IsMine(const CKeyStore& ks, const CScript& script) {
    std::vector<std::vector<unsigned char>> sol;
    txnouttype type;
    Solver(script, type, sol);
    switch (type) {
    case TX_NONSTANDARD:
    case TX_NULL_DATA: break;
    case TX_PUBKEY: {
        const CKeyID id = CPubKey(sol[0].begin(), sol[0].end()).GetID();
        if (ks.HaveKey(id)) return ISMINE_SPENDABLE;
        break;
    }
    case TX_PUBKEYHASH: {
        const CKeyID id{uint160(sol[0])};
        if (ks.HaveKey(id)) return ISMINE_SPENDABLE;
        break;
    }
    case TX_SCRIPTHASH: {
        const CScriptID id{uint160(sol[0])};
        CScript sub;
        if (ks.GetCScript(id, sub)) {
            const isminetype r = IsMine(ks, sub);
            if (r == ISMINE_SPENDABLE) return r;
        }
        break;
    }
    case TX_MULTISIG: {
        // only spendable when every key is ours (no partial multisig ownership)
        bool all = true;
        for (size_t i = 1; i + 1 < sol.size(); i++)
            if (!ks.HaveKey(CPubKey(sol[i].begin(), sol[i].end()).GetID())) all = false;
        if (all) return ISMINE_SPENDABLE;
        break;
    }
    }
    if (ks.HaveWatchOnly(script)) {
        SignatureData sd;
        return ProduceSignature(DummySignatureCreator(&ks), script, sd) ? ISMINE_WATCH_SOLVABLE
                                                                          : ISMINE_WATCH_UNSOLVABLE;
    }
    return ISMINE_NO;
}

isminetype IsMine(const CKeyStore& ks, const CTxDestination& dest) { return IsMine(ks, GetScriptForDestination(dest)); }

WalletLock::WalletLock(const CWallet& w) {
    if (w.chainstate) m = std::unique_lock<CCriticalSection>(w.chainstate->cs());
    l = std::unique_lock<CCriticalSection>(w.cs_wallet);
}

// ------------------------------------------------------------------ CWalletTx
int CWalletTx::GetDepthInMainChain(const CBlockIndex** ppindex) const {
    if (hashBlock.IsNull() || IsAbandoned() || !pwallet || !pwallet->chainstate) return 0;
    Chainstate& cs = *pwallet->chainstate;
    std::lock_guard<CCriticalSection> l(cs.cs());
    const CBlockIndex* pi = cs.LookupBlockIndex(hashBlock);
    if (!pi || !cs.ActiveChain().Contains(pi)) return 0;
    if (ppindex) *ppindex = pi;
    const int depth = cs.Height() - pi->nHeight + 1;
    return nIndex == -1 ? -depth : depth;
}

int CWalletTx::GetBlocksToMaturity() const {
    if (!IsCoinBase()) return 0;
    return std::max(0, (COINBASE_MATURITY + 1) - GetDepthInMainChain());
}

bool CWalletTx::InMempool() const { return pwallet && pwallet->mempool && pwallet->mempool->exists(GetHash()); }

bool CWalletTx::IsTrusted() const {
    if (!IsFinalTx(*tx, pwallet && pwallet->chainstate ? pwallet->chainstate->HeightNow() + 1 : 0, GetAdjustedTime()))
        return false;
    const int depth = GetDepthInMainChain();
    if (depth >= 1) return true;
    if (depth < 0) return false;
    if (!gArgs.GetBoolArg("-spendzeroconfchange", DEFAULT_SPEND_ZEROCONF_CHANGE) || !IsFromMe(ISMINE_ALL)) return false;
    if (!InMempool()) return false;
    for (const CTxIn& in : tx->vin) {
        const CWalletTx* parent = pwallet->GetWalletTx(in.prevout.hash);
        if (!parent) return false;
        if (pwallet->IsMine(parent->tx->vout[in.prevout.n]) != ISMINE_SPENDABLE) return false;
    }
    return true;
}

Amount CWalletTx::GetDebit(const isminefilter& filter) const {
    if (tx->vin.empty()) return 0;
    return pwallet->GetDebit(*tx, filter);
}

Amount CWalletTx::GetCredit(const isminefilter& filter) const {
    if (IsCoinBase() && GetBlocksToMaturity() > 0) return 0;
    return pwallet->GetCredit(*tx, filter);
}

Amount CWalletTx::GetImmatureCredit(bool) const {
    if (IsCoinBase() && GetBlocksToMaturity() > 0 && IsInMainChain()) return pwallet->GetCredit(*tx, ISMINE_SPENDABLE);
    return 0;
}

Amount CWalletTx::GetImmatureWatchOnlyCredit() const {
    if (IsCoinBase() && GetBlocksToMaturity() > 0 && IsInMainChain()) return pwallet->GetCredit(*tx, ISMINE_WATCH_ONLY);
    return 0;
}

Amount CWalletTx::GetAvailableCredit(bool) const {
    if (!pwallet) return 0;
    if (IsCoinBase() && GetBlocksToMaturity() > 0) return 0;
    Amount n = 0;
    for (unsigned i = 0; i < tx->vout.size(); i++)
        if (!pwallet->IsSpent(GetHash(), i)) n += pwallet->GetCredit(tx->vout[i], ISMINE_SPENDABLE);
    return n;
}

Amount CWalletTx::GetAvailableWatchOnlyCredit() const {
    if (!pwallet) return 0;
    if (IsCoinBase() && GetBlocksToMaturity() > 0) return 0;
    Amount n = 0;
    for (unsigned i = 0; i < tx->vout.size(); i++)
        if (!pwallet->IsSpent(GetHash(), i)) n += pwallet->GetCredit(tx->vout[i], ISMINE_WATCH_ONLY);
    return n;
}

Amount CWalletTx::GetChange() const {
    Amount n = 0;
    for (const CTxOut& o : tx->vout) n += pwallet->GetChange(o);
    return n;
}

bool CWalletTx::IsEquivalentTo(const CWalletTx& o) const {
    CMutableTransaction a(*tx), b(*o.tx);
    for (auto& in : a.vin) in.scriptSig = CScript();
    for (auto& in : b.vin) in.scriptSig = CScript();
    return CTransaction(a) == CTransaction(b);
}

void CWalletTx::GetAmounts(std::list<COutputEntry>& listReceived, std::list<COutputEntry>& listSent, Amount& nFee,
                           std::string& strSentAccount, const isminefilter& filter) const {
    nFee = 0;
    listReceived.clear();
    listSent.clear();
    strSentAccount = strFromAccount;
    const Amount nDebit = GetDebit(filter);
    if (nDebit > 0) nFee = nDebit - tx->GetValueOut();
    for (unsigned i = 0; i < tx->vout.size(); i++) {
        const CTxOut& out = tx->vout[i];
        const isminetype fIsMine = pwallet->IsMine(out);
        if (nDebit > 0) {
            if (pwallet->IsChange(out)) continue;
        } else if (!(fIsMine & filter)) {
            continue;
        }
        CTxDestination dest;
        if (!ExtractDestination(out.scriptPubKey, dest) && !out.scriptPubKey.IsUnspendable())
            LogPrintf("CWalletTx::GetAmounts: Unknown transaction type found, txid %s\n", GetHash().ToString().c_str());
        const COutputEntry e{dest, out.nValue, (int)i};
        if (nDebit > 0) listSent.push_back(e);
        if (fIsMine & filter) listReceived.push_back(e);
    }
}

std::set<uint256> CWalletTx::GetConflicts() const {
    std::set<uint256> result;
    if (!pwallet) return result;
    for (const CTxIn& in : tx->vin) {
        auto range = pwallet->mapTxSpends.equal_range(in.prevout);
        for (auto it = range.first; it != range.second; ++it)
            if (it->second != GetHash()) result.insert(it->second);
    }
    return result;
}

bool CWalletTx::RelayWalletTransaction() {
    if (IsCoinBase() || IsAbandoned() || GetDepthInMainChain() != 0) return false;
    if (!InMempool()) return false;
    LogPrintf("Relaying wtx %s\n", GetHash().ToString().c_str());
    if (g_relayTransaction) g_relayTransaction(GetHash());
    return true;
}

// ------------------------------------------------------------------ CReserveKey
bool CReserveKey::GetReservedKey(CPubKey& pubkey) {
    if (nIndex == -1) {
        CKeyPool kp;
        pwallet->ReserveKeyFromKeyPool(nIndex, kp);
        if (nIndex == -1) return false;
        vchPubKey = kp.vchPubKey;
    }
    pubkey = vchPubKey;
    return true;
}
void CReserveKey::KeepKey() {
    if (nIndex != -1) pwallet->KeepKey(nIndex);
    nIndex = -1;
    vchPubKey = CPubKey();
}
void CReserveKey::ReturnKey() {
    if (nIndex != -1) pwallet->ReturnKey(nIndex);
    nIndex = -1;
    vchPubKey = CPubKey();
}

// ------------------------------------------------------------------ CWallet
// -dblogsize: megabytes of wallet writes kept in the store's log before they are written out as
// a segment (the reference's Berkeley DB log size, wallet/db.cpp:319)
static KVOptions WalletStoreOptions() {
    KVOptions o;
    o.memtableBytes = (size_t)std::max<int64_t>(1, gArgs.GetArg("-dblogsize", (int64_t)100)) << 20;
    return o;
}

CWallet::CWallet(const std::string& name, const std::string& path, bool memoryOnly)
    : strWalletName(name), strWalletPath(path), db(new KVStore(path, memoryOnly, false, WalletStoreOptions())) {
    std::lock_guard<std::mutex> l(cs_wallets);
    g_wallets.push_back(this);
}

CWallet::~CWallet() {
    std::lock_guard<std::mutex> l(cs_wallets);
    g_wallets.erase(std::remove(g_wallets.begin(), g_wallets.end(), this), g_wallets.end());
}

void CWallet::Flush() { db->Write(std::string("orderposnext"), nOrderPosNext, true); }

void CWallet::FlushIfDirty() {
    WalletLock l(*this);
    const uint64_t b = db->LogBytes();
    if (b == nLastFlushBytes) return;
    Flush();
    nLastFlushBytes = db->LogBytes();
}

void CWallet::SetMinVersion(int v) {
    WalletLock l(*this);
    if (nWalletVersion >= v) return;
    nWalletVersion = v;
    if (v > nWalletMaxVersion) nWalletMaxVersion = v;
    db->Write(std::string("minversion"), v, true);
}

bool CWallet::Load(std::string& err, bool& firstRun) {
    WalletLock l(*this);
    firstRun = db->IsEmpty();
    KVIterator it(db.get());
    it.SeekToFirst();
    int nKeys = 0, nCKeys = 0, nTx = 0;
    std::map<CPubKey, std::vector<unsigned char>> pendingCrypted;
    for (; it.Valid(); it.Next()) {
        const std::string& raw = it.RawKey();
        std::string type;
        SpanReader r((const unsigned char*)raw.data(), raw.size(), SER_DISK, PROTOCOL_VERSION);
        try {
            r >> type;
            if (type == "name" || type == "purpose") {
                DestKey dk;
                r >> dk;
                std::string v;
                it.GetValue(v);
                if (type == "name") mapAddressBook[dk.d].name = v;
                else mapAddressBook[dk.d].purpose = v;
            } else if (type == "destdata") {
                std::pair<DestKey, std::string> k;
                r >> k;
                std::string v;
                it.GetValue(v);
                mapAddressBook[k.first.d].destdata[k.second] = v;
            } else if (type == "tx") {
                uint256 h;
                r >> h;
                CWalletTx wtx;
                if (!it.GetValue(wtx)) continue;
                wtx.pwallet = this;
                if (wtx.GetHash() != h) continue;
                mapWallet[h] = wtx;
                nTx++;
            } else if (type == "key") {
                CPubKey pub;
                r >> pub;
                CPrivKey priv; // locked memory, cleansed when freed
                it.GetValue(priv);
                CKey key;
                key.Set(priv.begin(), priv.end(), pub.IsCompressed());
                if (!key.IsValid() || !key.VerifyPubKey(pub)) {
                    err = "Error reading wallet database: private key corrupt";
                    return false;
                }
                LoadKey(key, pub);
                nKeys++;
            } else if (type == "ckey") {
                CPubKey pub;
                r >> pub;
                std::vector<unsigned char> c;
                it.GetValue(c);
                pendingCrypted[pub] = c;
                nCKeys++;
            } else if (type == "keymeta") {
                CPubKey pub;
                r >> pub;
                CKeyMetadata m;
                it.GetValue(m);
                mapKeyMetadata[pub.GetID()] = m;
                UpdateTimeFirstKey(m.nCreateTime);
            } else if (type == "watchmeta") {
                CScript s;
                r >> s;
                CKeyMetadata m;
                it.GetValue(m);
                mapScriptMetadata[CScriptID(s)] = m;
                UpdateTimeFirstKey(m.nCreateTime);
            } else if (type == "mkey") {
                unsigned int id;
                r >> id;
                CMasterKey mk;
                it.GetValue(mk);
                mapMasterKeys[id] = mk;
                nMasterKeyMaxID = std::max(nMasterKeyMaxID, id);
            } else if (type == "cscript") {
                CScriptID id;
                r >> id;
                CScript s;
                it.GetValue(s);
                CBasicKeyStore::AddCScript(s);
            } else if (type == "watchs") {
                CScript s;
                r >> s;
                CBasicKeyStore::AddWatchOnly(s);
            } else if (type == "pool") {
                int64_t idx;
                r >> idx;
                setKeyPool.insert(idx);
            } else if (type == "hdchain") {
                it.GetValue(hdChain);
            } else if (type == "defaultkey") {
                it.GetValue(vchDefaultKey);
            } else if (type == "orderposnext") {
                it.GetValue(nOrderPosNext);
            } else if (type == "minversion") {
                it.GetValue(nWalletVersion);
                if (nWalletVersion > CLIENT_VERSION) {
                    err = "Error loading " + strWalletName + ": Wallet requires newer version of Bitcoin Cash Plus";
                    return false;
                }
                nWalletMaxVersion = std::max(nWalletMaxVersion, nWalletVersion);
            } else if (type == "acentry") {
                std::pair<std::string, uint64_t> k;
                r >> k;
                CAccountingEntry e;
                it.GetValue(e);
                e.nEntryNo = k.second;
                nAccountingEntryNumber = std::max(nAccountingEntryNumber, k.second + 1);
                laccentries.push_back(e);
            }
        } catch (const std::exception& e) {
            LogPrintf("Wallet: skipping unreadable record (%s)\n", e.what());
        }
    }
    for (const auto& kv : pendingCrypted) CCryptoKeyStore::AddCryptedKey(kv.first, kv.second);
    if (nWalletVersion == 0) nWalletVersion = nWalletMaxVersion = WALLET_FEATURE_BASE;
    // order index and spend map
    bool fAnyUnordered = false;
    for (auto& kv : mapWallet) {
        fAnyUnordered |= kv.second.nOrderPos == -1;
        AddToSpends(kv.first);
    }
    for (const CAccountingEntry& e : laccentries) fAnyUnordered |= e.nOrderPos == -1;
    if (fAnyUnordered && !ReorderTransactions()) {
        err = "Error loading " + strWalletName + ": cannot write the transaction order";
        return false;
    }
    wtxOrdered.clear();
    for (auto& kv : mapWallet) wtxOrdered.insert({kv.second.nOrderPos, TxPair(&kv.second, nullptr)});
    for (CAccountingEntry& e : laccentries) wtxOrdered.insert({e.nOrderPos, TxPair(nullptr, &e)});
    LogPrintf("Wallet %s: %d keys, %d encrypted keys, %d transactions, %zu pool keys\n", strWalletName.c_str(), nKeys,
              nCKeys, nTx, setKeyPool.size());
    return true;
}

// Copies the wallet store to `dest` (reference CWalletDBWrapper::Backup: a directory
// destination gets the wallet's file name inside it, and copying onto the live wallet itself
// fails).
bool CWallet::BackupWallet(const std::string& destIn) {
    namespace fs = std::filesystem;
    WalletLock l(*this);
    Flush();
    std::error_code ec;
    fs::path dest(destIn);
    if (fs::is_directory(dest, ec) && !fs::exists(dest / "MANIFEST", ec)) dest /= strWalletName;
    if (!strWalletPath.empty()) {
        const fs::path a = fs::weakly_canonical(dest, ec), b = fs::weakly_canonical(fs::path(strWalletPath), ec);
        if (a == b) {
            LogPrintf("BackupWallet: cannot back the wallet up onto itself (%s)\n", destIn.c_str());
            return false;
        }
    }
    try {
        KVStore out(dest.string(), false, true);
        KVBatch b;
        KVIterator it(db.get());
        for (it.SeekToFirst(); it.Valid(); it.Next()) {
            std::string v;
            if (it.RawValue(v)) b.WriteRaw(it.RawKey(), v);
        }
        return out.WriteBatch(b, true);
    } catch (const std::exception& e) {
        LogPrintf("BackupWallet: %s\n", e.what());
        return false;
    }
}

void CWallet::UpdateTimeFirstKey(int64_t nCreateTime) {
    if (nCreateTime <= 1) nTimeFirstKey = 1; // unknown creation time: rescan everything
    else if (!nTimeFirstKey || nCreateTime < nTimeFirstKey) nTimeFirstKey = nCreateTime;
}

bool CWallet::WriteKeyRecords(const CPubKey& pub, const CKey* key, const std::vector<unsigned char>* crypted) {
    KVBatch b;
    if (key) b.Write(K("key", pub), key->GetPrivKeyBytes());
    if (crypted) {
        b.Write(K("ckey", pub), *crypted);
        b.Erase(K("key", pub));
    }
    auto m = mapKeyMetadata.find(pub.GetID());
    if (m != mapKeyMetadata.end()) b.Write(K("keymeta", pub), m->second);
    return db->WriteBatch(b, true);
}

bool CWallet::AddKeyPubKey(const CKey& key, const CPubKey& pubkey) {
    WalletLock l(*this);
    if (!mapKeyMetadata.count(pubkey.GetID())) {
        CKeyMetadata m;
        m.nCreateTime = GetTime();
        mapKeyMetadata[pubkey.GetID()] = m;
    }
    UpdateTimeFirstKey(mapKeyMetadata[pubkey.GetID()].nCreateTime);
    if (!CCryptoKeyStore::AddKeyPubKey(key, pubkey)) return false;
    // a watch-only script for the same key is now spendable
    const CScript script = GetScriptForDestination(pubkey.GetID());
    if (CBasicKeyStore::HaveWatchOnly(script)) RemoveWatchOnly(script);
    if (!IsCrypted()) return WriteKeyRecords(pubkey, &key, nullptr);
    return true; // AddCryptedKey wrote the record
}

bool CWallet::AddCryptedKey(const CPubKey& pubkey, const std::vector<unsigned char>& crypted) {
    if (!CCryptoKeyStore::AddCryptedKey(pubkey, crypted)) return false;
    WalletLock l(*this);
    return WriteKeyRecords(pubkey, nullptr, &crypted);
}

bool CWallet::AddCScript(const CScript& redeemScript) {
    if (!CBasicKeyStore::AddCScript(redeemScript)) return false;
    return db->Write(K("cscript", CScriptID(redeemScript)), redeemScript, true);
}

bool CWallet::AddWatchOnly(const CScript& dest) {
    if (!CBasicKeyStore::AddWatchOnly(dest)) return false;
    const CKeyMetadata& m = mapScriptMetadata[CScriptID(dest)];
    UpdateTimeFirstKey(m.nCreateTime);
    KVBatch b;
    b.Write(K("watchmeta", dest), m);
    b.Write(K("watchs", dest), std::string("1"));
    return db->WriteBatch(b, true);
}

bool CWallet::AddWatchOnly(const CScript& dest, int64_t nCreateTime) {
    mapScriptMetadata[CScriptID(dest)].nCreateTime = nCreateTime;
    return AddWatchOnly(dest);
}

bool CWallet::RemoveWatchOnly(const CScript& dest) {
    WalletLock l(*this);
    if (!CBasicKeyStore::RemoveWatchOnly(dest)) return false;
    KVBatch b;
    b.Erase(K("watchs", dest));
    b.Erase(K("watchmeta", dest));
    return db->WriteBatch(b, true);
}

CPubKey CWallet::DeriveNewChildKey(CKeyMetadata& metadata, CKey& secret) {
    CKey masterKey;
    if (!GetKey(hdChain.masterKeyID, masterKey)) throw std::runtime_error("CWallet::DeriveNewChildKey: Master key not found");
    CExtKey master;
    master.SetMaster(masterKey.begin(), masterKey.size());
    CExtKey account, external, child;
    master.Derive(account, BIP32_HARDENED_KEY_LIMIT);        // m/0'
    account.Derive(external, BIP32_HARDENED_KEY_LIMIT);      // m/0'/0'
    do {
        external.Derive(child, hdChain.nExternalChainCounter | BIP32_HARDENED_KEY_LIMIT);
        metadata.hdKeypath = "m/0'/0'/" + std::to_string(hdChain.nExternalChainCounter) + "'";
        metadata.hdMasterKeyID = hdChain.masterKeyID;
        hdChain.nExternalChainCounter++;
    } while (HaveKey(child.key.GetPubKey().GetID()));
    secret = child.key;
    db->Write(std::string("hdchain"), hdChain, true);
    return secret.GetPubKey();
}

CPubKey CWallet::GenerateNewKey() {
    WalletLock l(*this);
    CKey secret;
    CKeyMetadata metadata;
    metadata.nCreateTime = GetTime();
    if (IsHDEnabled()) DeriveNewChildKey(metadata, secret);
    else secret.MakeNewKey(true);
    const CPubKey pub = secret.GetPubKey();
    mapKeyMetadata[pub.GetID()] = metadata;
    UpdateTimeFirstKey(metadata.nCreateTime);
    if (!AddKeyPubKey(secret, pub)) throw std::runtime_error("CWallet::GenerateNewKey: AddKey failed");
    return pub;
}

CPubKey CWallet::GenerateNewHDMasterKey() {
    CKey key;
    key.MakeNewKey(true);
    const int64_t nCreationTime = GetTime();
    CKeyMetadata metadata;
    metadata.nCreateTime = nCreationTime;
    const CPubKey pub = key.GetPubKey();
    metadata.hdKeypath = "m";
    metadata.hdMasterKeyID = pub.GetID();
    {
        WalletLock l(*this);
        mapKeyMetadata[pub.GetID()] = metadata;
        if (!AddKeyPubKey(key, pub)) throw std::runtime_error("CWallet::GenerateNewHDMasterKey: AddKeyPubKey failed");
    }
    return pub;
}

bool CWallet::SetHDMasterKey(const CPubKey& pub) {
    WalletLock l(*this);
    CHDChain c;
    c.masterKeyID = pub.GetID();
    hdChain = c;
    return db->Write(std::string("hdchain"), hdChain, true);
}

bool CWallet::NewKeyPool() {
    WalletLock l(*this);
    KVBatch b;
    for (int64_t i : setKeyPool) b.Erase(K("pool", i));
    db->WriteBatch(b, true);
    setKeyPool.clear();
    if (IsLocked()) return false;
    TopUpKeyPool();
    return true;
}

bool CWallet::TopUpKeyPool(unsigned int kpSize) {
    WalletLock l(*this);
    if (IsLocked()) return false;
    const unsigned int nTarget =
        kpSize > 0 ? kpSize : (unsigned int)std::max<int64_t>(gArgs.GetArg("-keypool", (int64_t)DEFAULT_KEYPOOL_SIZE), 0);
    while (setKeyPool.size() < nTarget + 1) {
        const int64_t nEnd = setKeyPool.empty() ? 1 : *setKeyPool.rbegin() + 1;
        CKeyPool kp;
        kp.nTime = GetTime();
        kp.vchPubKey = GenerateNewKey();
        if (!db->Write(K("pool", nEnd), kp)) throw std::runtime_error("TopUpKeyPool(): writing generated key failed");
        setKeyPool.insert(nEnd);
    }
    return true;
}

void CWallet::ReserveKeyFromKeyPool(int64_t& nIndex, CKeyPool& keypool) {
    nIndex = -1;
    keypool.vchPubKey = CPubKey();
    WalletLock l(*this);
    if (!IsLocked()) TopUpKeyPool();
    if (setKeyPool.empty()) return;
    nIndex = *setKeyPool.begin();
    setKeyPool.erase(setKeyPool.begin());
    if (!db->Read(K("pool", nIndex), keypool)) throw std::runtime_error("ReserveKeyFromKeyPool(): read failed");
    if (!HaveKey(keypool.vchPubKey.GetID())) throw std::runtime_error("ReserveKeyFromKeyPool(): unknown key in key pool");
}

void CWallet::KeepKey(int64_t nIndex) { db->Erase(K("pool", nIndex)); }

void CWallet::ReturnKey(int64_t nIndex) {
    WalletLock l(*this);
    setKeyPool.insert(nIndex);
}

bool CWallet::GetKeyFromPool(CPubKey& result) {
    WalletLock l(*this);
    int64_t nIndex = 0;
    CKeyPool kp;
    ReserveKeyFromKeyPool(nIndex, kp);
    if (nIndex == -1) {
        if (IsLocked()) return false;
        result = GenerateNewKey();
        return true;
    }
    KeepKey(nIndex);
    result = kp.vchPubKey;
    return true;
}

int64_t CWallet::GetOldestKeyPoolTime() {
    WalletLock l(*this);
    if (setKeyPool.empty()) return GetTime();
    CKeyPool kp;
    if (!db->Read(K("pool", *setKeyPool.begin()), kp)) return GetTime();
    return kp.nTime;
}

bool CWallet::EncryptWallet(const std::string& passphrase) {
    if (IsCrypted()) return false;
    CKeyingMaterial masterKey(WALLET_CRYPTO_KEY_SIZE);
    GetStrongRandBytes(masterKey.data(), WALLET_CRYPTO_KEY_SIZE);
    CMasterKey mk;
    mk.vchSalt.resize(WALLET_CRYPTO_SALT_SIZE);
    GetStrongRandBytes(mk.vchSalt.data(), WALLET_CRYPTO_SALT_SIZE);
    // calibrate the derivation to ~100 ms (reference crypter iteration tuning)
    CCrypter crypter;
    int64_t t0 = GetTimeMillis();
    crypter.SetKeyFromPassphrase(passphrase, mk.vchSalt, 25000, 0);
    const int64_t dt = std::max<int64_t>(1, GetTimeMillis() - t0);
    mk.nDeriveIterations = (unsigned int)std::max<int64_t>(25000, 25000 * 100 / dt);
    if (!crypter.SetKeyFromPassphrase(passphrase, mk.vchSalt, mk.nDeriveIterations, mk.nDerivationMethod)) return false;
    if (!crypter.Encrypt(masterKey, mk.vchCryptedKey)) return false;
    {
        WalletLock l(*this);
        mapMasterKeys[++nMasterKeyMaxID] = mk;
        db->Write(K("mkey", nMasterKeyMaxID), mk, true);
        std::set<CKeyID> plainIds;
        for (const auto& kv : mapKeys) plainIds.insert(kv.first);
        if (!EncryptKeys(masterKey)) throw std::runtime_error("EncryptWallet: key encryption failed");
        KVBatch b;
        for (const auto& kv : mapCryptedKeys) {
            b.Write(K("ckey", kv.second.first), kv.second.second);
            b.Erase(K("key", kv.second.first));
        }
        db->WriteBatch(b, true);
        SetMinVersion(WALLET_FEATURE_WALLETCRYPT);
        Lock();
        Unlock(passphrase);
        // fresh HD seed and key pool: the old ones were written unencrypted
        if (IsHDEnabled()) SetHDMasterKey(GenerateNewHDMasterKey());
        NewKeyPool();
        Lock();
    }
    return true;
}

bool CWallet::Unlock(const std::string& passphrase) {
    CCrypter crypter;
    CKeyingMaterial masterKey;
    WalletLock l(*this);
    for (const auto& kv : mapMasterKeys) {
        if (!crypter.SetKeyFromPassphrase(passphrase, kv.second.vchSalt, kv.second.nDeriveIterations,
                                          kv.second.nDerivationMethod))
            return false;
        if (!crypter.Decrypt(kv.second.vchCryptedKey, masterKey)) continue;
        if (CCryptoKeyStore::Unlock(masterKey)) return true;
    }
    return false;
}

bool CWallet::ChangeWalletPassphrase(const std::string& oldPass, const std::string& newPass) {
    const bool wasLocked = IsLocked();
    WalletLock l(*this);
    Lock();
    CCrypter crypter;
    CKeyingMaterial masterKey;
    for (auto& kv : mapMasterKeys) {
        if (!crypter.SetKeyFromPassphrase(oldPass, kv.second.vchSalt, kv.second.nDeriveIterations,
                                          kv.second.nDerivationMethod))
            return false;
        if (!crypter.Decrypt(kv.second.vchCryptedKey, masterKey)) return false;
        if (CCryptoKeyStore::Unlock(masterKey)) {
            if (!crypter.SetKeyFromPassphrase(newPass, kv.second.vchSalt, kv.second.nDeriveIterations,
                                              kv.second.nDerivationMethod))
                return false;
            if (!crypter.Encrypt(masterKey, kv.second.vchCryptedKey)) return false;
            db->Write(K("mkey", kv.first), kv.second, true);
            if (wasLocked) Lock();
            return true;
        }
    }
    return false;
}

// ------------------------------------------------------------------ tx bookkeeping
int64_t CWallet::IncOrderPosNext() {
    const int64_t r = nOrderPosNext++;
    db->Write(std::string("orderposnext"), nOrderPosNext);
    return r;
}

const CWalletTx* CWallet::GetWalletTx(const uint256& hash) const {
    WalletLock l(*this);
    auto it = mapWallet.find(hash);
    return it == mapWallet.end() ? nullptr : &it->second;
}

void CWallet::AddToSpends(const COutPoint& outpoint, const uint256& wtxid) {
    mapTxSpends.insert({outpoint, wtxid});
    SyncMetaData(outpoint);
}

// Wallet transactions that spend the same outpoint and differ only in their signatures (a
// malleated copy, or a clone signed with another hash type) share the oldest one's metadata:
// comments, order form, smart time, from-me and the account it was sent from (reference
// wallet.cpp:590-634 SyncMetaData).
void CWallet::SyncMetaData(const COutPoint& outpoint) {
    auto range = mapTxSpends.equal_range(outpoint);
    const CWalletTx* copyFrom = nullptr;
    int64_t minOrder = std::numeric_limits<int64_t>::max();
    for (auto it = range.first; it != range.second; ++it) {
        auto mit = mapWallet.find(it->second);
        if (mit != mapWallet.end() && mit->second.nOrderPos < minOrder) {
            minOrder = mit->second.nOrderPos;
            copyFrom = &mit->second;
        }
    }
    if (!copyFrom) return;
    for (auto it = range.first; it != range.second; ++it) {
        auto mit = mapWallet.find(it->second);
        if (mit == mapWallet.end()) continue;
        CWalletTx* copyTo = &mit->second;
        if (copyTo == copyFrom || !copyFrom->IsEquivalentTo(*copyTo)) continue;
        copyTo->mapValue = copyFrom->mapValue;
        copyTo->vOrderForm = copyFrom->vOrderForm;
        copyTo->nTimeSmart = copyFrom->nTimeSmart; // nTimeReceived and nOrderPos stay the copy's own
        copyTo->fFromMe = copyFrom->fFromMe;
        copyTo->strFromAccount = copyFrom->strFromAccount;
    }
}

void CWallet::AddToSpends(const uint256& wtxid) {
    const CWalletTx& wtx = mapWallet.at(wtxid);
    if (wtx.IsCoinBase()) return;
    for (const CTxIn& in : wtx.tx->vin) AddToSpends(in.prevout, wtxid);
}

bool CWallet::IsSpent(const uint256& hash, unsigned int n) const {
    const COutPoint o(hash, n);
    auto range = mapTxSpends.equal_range(o);
    for (auto it = range.first; it != range.second; ++it) {
        auto mit = mapWallet.find(it->second);
        if (mit != mapWallet.end()) {
            const int depth = mit->second.GetDepthInMainChain();
            if (depth > 0 || (depth == 0 && !mit->second.IsAbandoned())) return true;
        }
    }
    return false;
}

bool CWallet::AddToWallet(const CWalletTx& wtxIn, bool) {
    WalletLock l(*this);
    const uint256 hash = wtxIn.GetHash();
    auto ret = mapWallet.insert({hash, wtxIn});
    CWalletTx& wtx = ret.first->second;
    wtx.pwallet = this;
    const bool fInsertedNew = ret.second;
    bool fUpdated = false;
    if (fInsertedNew) {
        wtx.nTimeReceived = (uint32_t)GetAdjustedTime();
        wtx.nOrderPos = IncOrderPosNext();
        wtxOrdered.insert({wtx.nOrderPos, TxPair(&wtx, nullptr)});
        // smart time: block time for confirmed txs we learn about late, else receive time
        wtx.nTimeSmart = wtx.nTimeReceived;
        if (!wtxIn.hashBlock.IsNull() && !wtxIn.IsAbandoned() && chainstate) {
            const CBlockIndex* pi = chainstate->LookupBlockIndex(wtxIn.hashBlock);
            if (pi) wtx.nTimeSmart = (uint32_t)std::min<int64_t>(pi->GetBlockTime(), wtx.nTimeReceived);
        }
        AddToSpends(hash);
    } else {
        if (!wtxIn.hashBlock.IsNull() && wtxIn.hashBlock != wtx.hashBlock) {
            wtx.hashBlock = wtxIn.hashBlock;
            fUpdated = true;
        }
        if (wtxIn.nIndex != -1 && wtxIn.nIndex != wtx.nIndex) {
            wtx.nIndex = wtxIn.nIndex;
            fUpdated = true;
        }
        if (wtxIn.fFromMe && wtxIn.fFromMe != wtx.fFromMe) {
            wtx.fFromMe = wtxIn.fFromMe;
            fUpdated = true;
        }
    }
    LogPrintf("AddToWallet %s  %s%s\n", hash.ToString().c_str(), fInsertedNew ? "new" : "", fUpdated ? "update" : "");
    if (fInsertedNew || fUpdated) db->Write(K("tx", hash), wtx);
    // -walletnotify=<cmd>: %s is replaced by the txid
    const std::string cmd = gArgs.GetArg("-walletnotify", "");
    if (!cmd.empty() && (fInsertedNew || fUpdated)) {
        std::string c = cmd;
        ReplaceAll(c, "%s", hash.GetHex());
        RunCommandAsync(c);
    }
    return true;
}

bool CWallet::AddToWalletIfInvolvingMe(const CTransactionRef& ptx, const CBlockIndex* pIndex, int posInBlock,
                                       bool fUpdate) {
    const CTransaction& tx = *ptx;
    WalletLock l(*this);
    if (pIndex) {
        for (const CTxIn& in : tx.vin) {
            auto range = mapTxSpends.equal_range(in.prevout);
            std::vector<uint256> others;
            for (auto it = range.first; it != range.second; ++it)
                if (it->second != tx.GetHash()) others.push_back(it->second);
            for (const uint256& o : others) MarkConflicted(pIndex->GetBlockHash(), o);
        }
    }
    const bool fExisted = mapWallet.count(tx.GetHash()) != 0;
    if (fExisted && !fUpdate) return false;
    if (fExisted || IsMine(tx) || IsFromMe(tx)) {
        CWalletTx wtx(this, ptx);
        if (pIndex) {
            wtx.hashBlock = pIndex->GetBlockHash();
            wtx.nIndex = posInBlock;
        }
        return AddToWallet(wtx, false);
    }
    return false;
}

bool CWallet::MarkConflicted(const uint256& hashBlock, const uint256& hashTx) {
    WalletLock l(*this);
    const CBlockIndex* pi = chainstate ? chainstate->LookupBlockIndex(hashBlock) : nullptr;
    if (!pi) return false;
    std::set<uint256> todo{hashTx}, done;
    while (!todo.empty()) {
        const uint256 now = *todo.begin();
        todo.erase(todo.begin());
        done.insert(now);
        auto it = mapWallet.find(now);
        if (it == mapWallet.end()) continue;
        CWalletTx& wtx = it->second;
        if (wtx.GetDepthInMainChain() > 0) continue;
        wtx.nIndex = -1;
        wtx.hashBlock = hashBlock;
        db->Write(K("tx", now), wtx);
        for (unsigned i = 0; i < wtx.tx->vout.size(); i++) {
            auto range = mapTxSpends.equal_range(COutPoint(now, i));
            for (auto s = range.first; s != range.second; ++s)
                if (!done.count(s->second)) todo.insert(s->second);
        }
    }
    return true;
}

bool CWallet::AbandonTransaction(const uint256& hashTx) {
    WalletLock l(*this);
    auto it = mapWallet.find(hashTx);
    if (it == mapWallet.end()) return false;
    if (it->second.GetDepthInMainChain() != 0 || it->second.InMempool()) return false;
    std::set<uint256> todo{hashTx}, done;
    while (!todo.empty()) {
        const uint256 now = *todo.begin();
        todo.erase(todo.begin());
        done.insert(now);
        auto wit = mapWallet.find(now);
        if (wit == mapWallet.end()) continue;
        CWalletTx& wtx = wit->second;
        if (wtx.GetDepthInMainChain() != 0) continue;
        if (!wtx.IsAbandoned()) {
            wtx.SetAbandoned();
            db->Write(K("tx", now), wtx);
        }
        for (unsigned i = 0; i < wtx.tx->vout.size(); i++) {
            auto range = mapTxSpends.equal_range(COutPoint(now, i));
            for (auto s = range.first; s != range.second; ++s)
                if (!done.count(s->second)) todo.insert(s->second);
        }
    }
    return true;
}

void CWallet::SyncTransaction(const CTransactionRef& tx, const CBlockIndex* pindex, int posInBlock) {
    WalletLock l(*this);
    AddToWalletIfInvolvingMe(tx, pindex, posInBlock, true);
}

void CWallet::TransactionAddedToMempool(const CTransactionRef& tx) { SyncTransaction(tx); }

void CWallet::BlockConnected(const std::shared_ptr<const CBlock>& block, const CBlockIndex* pindex,
                             const std::vector<CTransactionRef>& conflicted) {
    WalletLock l(*this);
    for (const CTransactionRef& t : conflicted) SyncTransaction(t);
    for (size_t i = 0; i < block->vtx.size(); i++) SyncTransaction(block->vtx[i], pindex, (int)i);
}

void CWallet::BlockDisconnected(const std::shared_ptr<const CBlock>& block) {
    WalletLock l(*this);
    for (const CTransactionRef& t : block->vtx) SyncTransaction(t);
}

void CWallet::SetBestChain(const CBlockLocator& loc) { db->Write(std::string("bestblock"), loc); }

std::vector<uint256> CWallet::ResendWalletTransactionsBefore(int64_t nTime) {
    std::vector<uint256> result;
    WalletLock l(*this);
    std::multimap<unsigned int, CWalletTx*> sorted;
    for (auto& kv : mapWallet) {
        if (kv.second.nTimeReceived > nTime) continue;
        sorted.insert({kv.second.nTimeReceived, &kv.second});
    }
    for (auto& kv : sorted)
        if (kv.second->RelayWalletTransaction()) result.push_back(kv.second->GetHash());
    return result;
}

void CWallet::ResendWalletTransactions(int64_t nBestBlockTime) {
    // randomised schedule so the resend doesn't fingerprint the wallet
    if (GetTime() < nNextResend || !fBroadcastTransactions) return;
    const bool fFirst = nNextResend == 0;
    nNextResend = GetTime() + GetRand(30 * 60);
    if (fFirst) return;
    if (nBestBlockTime < nLastResend) return;
    nLastResend = GetTime();
    const std::vector<uint256> r = ResendWalletTransactionsBefore(nBestBlockTime - 5 * 60);
    if (!r.empty()) LogPrintf("%s: rebroadcast %zu unconfirmed transactions\n", __func__, r.size());
}

void CWallet::ReacceptWalletTransactions() {
    if (!fBroadcastTransactions || !chainstate) return;
    std::lock_guard<CCriticalSection> lm(chainstate->cs());
    WalletLock l(*this);
    std::map<int64_t, CWalletTx*> mapSorted;
    for (auto& kv : mapWallet) {
        CWalletTx& wtx = kv.second;
        if (!wtx.IsCoinBase() && wtx.GetDepthInMainChain() == 0 && !wtx.IsAbandoned())
            mapSorted.insert({wtx.nOrderPos, &wtx});
    }
    for (auto& kv : mapSorted) {
        CValidationState st;
        chainstate->AcceptToMemoryPool(st, kv.second->tx, false, nullptr);
    }
}

bool CWallet::ScanForWalletTransactions(const CBlockIndex* pindex, bool fUpdate, int* pnFound) {
    if (!chainstate) return false;
    int found = 0;
    const int64_t start = GetTimeMillis();
    int tipHeight = 0;
    {
        std::lock_guard<CCriticalSection> lm(chainstate->cs());
        tipHeight = std::max(1, chainstate->Height());
    }
    const int firstHeight = pindex ? pindex->nHeight : 0;
    uiInterface.ShowProgress("Rescanning...", 0);
    while (pindex) {
        if (pindex->nHeight % 100 == 0)
            uiInterface.ShowProgress("Rescanning...",
                                     std::max(1, std::min(99, (int)(100.0 * (pindex->nHeight - firstHeight) /
                                                                    std::max(1, tipHeight - firstHeight)))));
        CBlock block;
        {
            std::lock_guard<CCriticalSection> lm(chainstate->cs());
            if (!chainstate->ReadBlock(block, pindex, false)) break;
            WalletLock l(*this);
            for (size_t i = 0; i < block.vtx.size(); i++)
                if (AddToWalletIfInvolvingMe(block.vtx[i], pindex, (int)i, fUpdate)) found++;
            pindex = chainstate->ActiveChain().Next(pindex);
        }
    }
    uiInterface.ShowProgress("Rescanning...", 100);
    if (pnFound) *pnFound = found;
    LogPrintf("Rescan completed in %15dms (%d wallet txs)\n", (int)(GetTimeMillis() - start), found);
    return true;
}

bool CWallet::ReorderTransactions() {
    WalletLock l(*this);
    // everything by time; equal times keep the order they were gathered in
    std::multimap<int64_t, TxPair> txByTime;
    for (auto& kv : mapWallet) txByTime.insert({(int64_t)kv.second.nTimeReceived, TxPair(&kv.second, nullptr)});
    // the reference reads the entries with ListAccountCreditDebit(""): account "" only
    for (CAccountingEntry& e : laccentries)
        if (e.strAccount.empty()) txByTime.insert({e.nTime, TxPair(nullptr, &e)});
    nOrderPosNext = 0;
    std::vector<int64_t> offsets; // positions handed to unordered records, in increasing order
    for (auto& it : txByTime) {
        CWalletTx* const pwtx = it.second.first;
        CAccountingEntry* const pae = it.second.second;
        int64_t& pos = pwtx ? pwtx->nOrderPos : pae->nOrderPos;
        if (pos == -1) {
            pos = nOrderPosNext++;
            offsets.push_back(pos);
        } else {
            int64_t off = 0;
            for (int64_t start : offsets)
                if (pos >= start) ++off;
            pos += off;
            nOrderPosNext = std::max(nOrderPosNext, pos + 1);
            if (!off) continue;
        }
        const bool ok = pwtx ? db->Write(K("tx", pwtx->GetHash()), *pwtx)
                             : db->Write(K("acentry", std::make_pair(pae->strAccount, pae->nEntryNo)), *pae);
        if (!ok) return false;
    }
    db->Write(std::string("orderposnext"), nOrderPosNext);
    wtxOrdered.clear();
    for (auto& kv : mapWallet) wtxOrdered.insert({kv.second.nOrderPos, TxPair(&kv.second, nullptr)});
    for (CAccountingEntry& e : laccentries) wtxOrdered.insert({e.nOrderPos, TxPair(nullptr, &e)});
    return true;
}

bool CWallet::AddAccountingEntry(const CAccountingEntry& entryIn) {
    WalletLock l(*this);
    CAccountingEntry e = entryIn;
    e.nEntryNo = nAccountingEntryNumber++;
    if (!db->Write(K("acentry", std::make_pair(e.strAccount, e.nEntryNo)), e)) return false;
    laccentries.push_back(e);
    CAccountingEntry& stored = laccentries.back();
    wtxOrdered.insert({stored.nOrderPos, TxPair(nullptr, &stored)});
    return true;
}

// ------------------------------------------------------------------ ownership
isminetype CWallet::IsMine(const CTxIn& txin) const {
    WalletLock l(*this);
    auto it = mapWallet.find(txin.prevout.hash);
    if (it != mapWallet.end() && txin.prevout.n < it->second.tx->vout.size())
        return IsMine(it->second.tx->vout[txin.prevout.n]);
    return ISMINE_NO;
}
isminetype CWallet::IsMine(const CTxOut& txout) const { return ::bcp::IsMine(*this, txout.scriptPubKey); }
bool CWallet::IsMine(const CTransaction& tx) const {
    for (const CTxOut& o : tx.vout)
        if (IsMine(o)) return true;
    return false;
}
bool CWallet::IsFromMe(const CTransaction& tx) const { return GetDebit(tx, ISMINE_ALL) > 0; }

Amount CWallet::GetDebit(const CTxIn& txin, const isminefilter& filter) const {
    WalletLock l(*this);
    auto it = mapWallet.find(txin.prevout.hash);
    if (it != mapWallet.end() && txin.prevout.n < it->second.tx->vout.size())
        if (IsMine(it->second.tx->vout[txin.prevout.n]) & filter) return it->second.tx->vout[txin.prevout.n].nValue;
    return 0;
}
Amount CWallet::GetDebit(const CTransaction& tx, const isminefilter& filter) const {
    Amount n = 0;
    for (const CTxIn& in : tx.vin) n += GetDebit(in, filter);
    return n;
}
Amount CWallet::GetCredit(const CTxOut& txout, const isminefilter& filter) const {
    return (IsMine(txout) & filter) ? txout.nValue : 0;
}
Amount CWallet::GetCredit(const CTransaction& tx, const isminefilter& filter) const {
    Amount n = 0;
    for (const CTxOut& o : tx.vout) n += GetCredit(o, filter);
    return n;
}
bool CWallet::IsChange(const CTxOut& txout) const {
    // mine, and the destination is not in the address book
    if (IsMine(txout)) {
        CTxDestination d;
        if (!ExtractDestination(txout.scriptPubKey, d)) return true;
        WalletLock l(*this);
        if (!mapAddressBook.count(d)) return true;
    }
    return false;
}
Amount CWallet::GetChange(const CTxOut& txout) const { return IsChange(txout) ? txout.nValue : 0; }

Amount CWallet::GetBalance() const {
    WalletLock l(*this);
    Amount n = 0;
    for (const auto& kv : mapWallet)
        if (kv.second.IsTrusted()) n += kv.second.GetAvailableCredit();
    return n;
}
Amount CWallet::GetUnconfirmedBalance() const {
    WalletLock l(*this);
    Amount n = 0;
    for (const auto& kv : mapWallet)
        if (!kv.second.IsTrusted() && kv.second.GetDepthInMainChain() == 0 && kv.second.InMempool())
            n += kv.second.GetAvailableCredit();
    return n;
}
Amount CWallet::GetImmatureBalance() const {
    WalletLock l(*this);
    Amount n = 0;
    for (const auto& kv : mapWallet) n += kv.second.GetImmatureCredit();
    return n;
}
Amount CWallet::GetWatchOnlyBalance() const {
    WalletLock l(*this);
    Amount n = 0;
    for (const auto& kv : mapWallet)
        if (kv.second.IsTrusted()) n += kv.second.GetAvailableWatchOnlyCredit();
    return n;
}
Amount CWallet::GetUnconfirmedWatchOnlyBalance() const {
    WalletLock l(*this);
    Amount n = 0;
    for (const auto& kv : mapWallet)
        if (!kv.second.IsTrusted() && kv.second.GetDepthInMainChain() == 0 && kv.second.InMempool())
            n += kv.second.GetAvailableWatchOnlyCredit();
    return n;
}
Amount CWallet::GetImmatureWatchOnlyBalance() const {
    WalletLock l(*this);
    Amount n = 0;
    for (const auto& kv : mapWallet) n += kv.second.GetImmatureWatchOnlyCredit();
    return n;
}

Amount CWallet::GetAccountBalance(const std::string& strAccount, int nMinDepth, const isminefilter& filter) {
    WalletLock l(*this);
    Amount nBalance = 0;
    for (const auto& kv : mapWallet) {
        const CWalletTx& wtx = kv.second;
        if (!IsFinalTx(*wtx.tx, chainstate ? chainstate->HeightNow() + 1 : 0, GetAdjustedTime()) ||
            wtx.GetBlocksToMaturity() > 0 || wtx.GetDepthInMainChain() < 0)
            continue;
        std::list<COutputEntry> received, sent;
        Amount fee = 0;
        std::string sentAccount;
        wtx.GetAmounts(received, sent, fee, sentAccount, filter);
        if (wtx.GetDepthInMainChain() >= nMinDepth) {
            for (const COutputEntry& r : received) {
                auto it = mapAddressBook.find(r.destination);
                const std::string acc = it == mapAddressBook.end() ? "" : it->second.name;
                if (acc == strAccount) nBalance += r.amount;
            }
        }
        if (sentAccount == strAccount) {
            for (const COutputEntry& s : sent) nBalance -= s.amount;
            nBalance -= fee;
        }
    }
    for (const CAccountingEntry& e : laccentries)
        if (e.strAccount == strAccount) nBalance += e.nCreditDebit;
    return nBalance;
}

std::set<CTxDestination> CWallet::GetAccountAddresses(const std::string& strAccount) const {
    WalletLock l(*this);
    std::set<CTxDestination> r;
    for (const auto& kv : mapAddressBook)
        if (kv.second.name == strAccount) r.insert(kv.first);
    return r;
}

std::map<CTxDestination, Amount> CWallet::GetAddressBalances() {
    std::map<CTxDestination, Amount> balances;
    WalletLock l(*this);
    for (const auto& kv : mapWallet) {
        const CWalletTx& wtx = kv.second;
        if (!wtx.IsTrusted()) continue;
        if (wtx.IsCoinBase() && wtx.GetBlocksToMaturity() > 0) continue;
        const int nDepth = wtx.GetDepthInMainChain();
        if (nDepth < (wtx.IsFromMe(ISMINE_ALL) ? 0 : 1)) continue;
        for (unsigned i = 0; i < wtx.tx->vout.size(); i++) {
            CTxDestination addr;
            if (!IsMine(wtx.tx->vout[i])) continue;
            if (!ExtractDestination(wtx.tx->vout[i].scriptPubKey, addr)) continue;
            const Amount n = IsSpent(kv.first, i) ? 0 : wtx.tx->vout[i].nValue;
            balances[addr] += n;
        }
    }
    return balances;
}

std::set<std::set<CTxDestination>> CWallet::GetAddressGroupings() {
    WalletLock l(*this);
    std::set<std::set<CTxDestination>> groupings;
    for (const auto& kv : mapWallet) {
        const CWalletTx& wtx = kv.second;
        std::set<CTxDestination> grouping;
        if (!wtx.tx->vin.empty()) {
            bool any_mine = false;
            for (const CTxIn& in : wtx.tx->vin) {
                CTxDestination addr;
                if (!IsMine(in)) continue;
                auto pit = mapWallet.find(in.prevout.hash);
                if (pit == mapWallet.end()) continue;
                if (!ExtractDestination(pit->second.tx->vout[in.prevout.n].scriptPubKey, addr)) continue;
                grouping.insert(addr);
                any_mine = true;
            }
            if (any_mine) {
                for (const CTxOut& o : wtx.tx->vout)
                    if (IsChange(o)) {
                        CTxDestination a;
                        if (ExtractDestination(o.scriptPubKey, a)) grouping.insert(a);
                    }
            }
            if (!grouping.empty()) {
                groupings.insert(grouping);
                grouping.clear();
            }
        }
        for (const CTxOut& o : wtx.tx->vout)
            if (IsMine(o)) {
                CTxDestination a;
                if (!ExtractDestination(o.scriptPubKey, a)) continue;
                grouping.insert(a);
                groupings.insert(grouping);
                grouping.clear();
            }
    }
    // merge overlapping groups (union-find over address sets)
    std::vector<std::set<CTxDestination>> merged;
    for (const auto& g : groupings) {
        std::set<CTxDestination> cur = g;
        for (auto it = merged.begin(); it != merged.end();) {
            bool overlap = false;
            for (const auto& a : cur)
                if (it->count(a)) {
                    overlap = true;
                    break;
                }
            if (overlap) {
                cur.insert(it->begin(), it->end());
                it = merged.erase(it);
            } else {
                ++it;
            }
        }
        merged.push_back(cur);
    }
    return std::set<std::set<CTxDestination>>(merged.begin(), merged.end());
}

// ------------------------------------------------------------------ coins
void CWallet::AvailableCoins(std::vector<COutput>& vCoins, bool fOnlyConfirmed, const CCoinControl* coinControl,
                             bool fIncludeZeroValue) const {
    vCoins.clear();
    WalletLock l(*this);
    const int height = chainstate ? chainstate->HeightNow() : 0; // (WalletLock holds cs_main already)
    for (const auto& kv : mapWallet) {
        const CWalletTx& wtx = kv.second;
        if (!IsFinalTx(*wtx.tx, height + 1, GetAdjustedTime())) continue;
        if (fOnlyConfirmed && !wtx.IsTrusted()) continue;
        if (wtx.IsCoinBase() && wtx.GetBlocksToMaturity() > 0) continue;
        const int nDepth = wtx.GetDepthInMainChain();
        if (nDepth < 0) continue;
        if (nDepth == 0 && !wtx.InMempool()) continue;
        for (unsigned i = 0; i < wtx.tx->vout.size(); i++) {
            const isminetype mine = IsMine(wtx.tx->vout[i]);
            if (IsSpent(kv.first, i) || mine == ISMINE_NO || IsLockedCoin(kv.first, i)) continue;
            if (wtx.tx->vout[i].nValue <= 0 && !fIncludeZeroValue) continue;
            if (coinControl && coinControl->HasSelected() && !coinControl->fAllowOtherInputs &&
                !coinControl->IsSelected(COutPoint(kv.first, i)))
                continue;
            const bool fSpendable = (mine & ISMINE_SPENDABLE) != ISMINE_NO ||
                                    (coinControl && coinControl->fAllowWatchOnly && (mine & ISMINE_WATCH_SOLVABLE));
            const bool fSolvable = (mine & (ISMINE_SPENDABLE | ISMINE_WATCH_SOLVABLE)) != ISMINE_NO;
            vCoins.push_back({&wtx, (int)i, nDepth, fSpendable, fSolvable});
        }
    }
}

// Randomised subset-sum search: repeatedly include coins at random (then
// deterministically) until the target is reached, keeping the smallest total >= target.
static void ApproximateBestSubset(const std::vector<std::pair<Amount, std::pair<const CWalletTx*, unsigned>>>& vValue,
                                  Amount nTotalLower, Amount nTargetValue, std::vector<char>& vfBest, Amount& nBest,
                                  int iterations = 1000) {
    std::vector<char> vfIncluded;
    vfBest.assign(vValue.size(), true);
    nBest = nTotalLower;
    FastRandomContext rng;
    for (int rep = 0; rep < iterations && nBest != nTargetValue; rep++) {
        vfIncluded.assign(vValue.size(), false);
        Amount nTotal = 0;
        bool fReachedTarget = false;
        for (int pass = 0; pass < 2 && !fReachedTarget; pass++) {
            for (size_t i = 0; i < vValue.size(); i++) {
                if (pass == 0 ? (rng.randbits(1) != 0) : !vfIncluded[i]) {
                    nTotal += vValue[i].first;
                    vfIncluded[i] = true;
                    if (nTotal >= nTargetValue) {
                        fReachedTarget = true;
                        if (nTotal < nBest) {
                            nBest = nTotal;
                            vfBest = vfIncluded;
                        }
                        nTotal -= vValue[i].first;
                        vfIncluded[i] = false;
                    }
                }
            }
        }
    }
}

bool CWallet::SelectCoinsMinConf(Amount nTargetValue, int nConfMine, int nConfTheirs, uint64_t nMaxAncestors, std::vector<COutput> vCoins,
                                 std::set<std::pair<const CWalletTx*, unsigned int>>& setCoinsRet,
                                 Amount& nValueRet) const {
    setCoinsRet.clear();
    nValueRet = 0;
    typedef std::pair<Amount, std::pair<const CWalletTx*, unsigned>> ValuedCoin;
    ValuedCoin coinLowestLarger{INT64_MAX, {nullptr, 0}};
    std::vector<ValuedCoin> vValue;
    Amount nTotalLower = 0;
    std::shuffle(vCoins.begin(), vCoins.end(), std::mt19937((unsigned)GetRand(UINT32_MAX)));
    for (const COutput& o : vCoins) {
        if (!o.fSpendable) continue;
        const CWalletTx* pcoin = o.tx;
        if (o.nDepth < (pcoin->IsFromMe(ISMINE_ALL) ? nConfMine : nConfTheirs)) continue;
        if (mempool && !mempool->TransactionWithinChainLimit(pcoin->GetHash(), nMaxAncestors)) continue;
        const Amount n = pcoin->tx->vout[o.i].nValue;
        const ValuedCoin coin{n, {pcoin, (unsigned)o.i}};
        if (n == nTargetValue) {
            setCoinsRet.insert(coin.second);
            nValueRet += n;
            return true;
        } else if (n < nTargetValue + MIN_CHANGE) {
            vValue.push_back(coin);
            nTotalLower += n;
        } else if (n < coinLowestLarger.first) {
            coinLowestLarger = coin;
        }
    }
    if (nTotalLower == nTargetValue) {
        for (const ValuedCoin& c : vValue) {
            setCoinsRet.insert(c.second);
            nValueRet += c.first;
        }
        return true;
    }
    if (nTotalLower < nTargetValue) {
        if (!coinLowestLarger.second.first) return false;
        setCoinsRet.insert(coinLowestLarger.second);
        nValueRet += coinLowestLarger.first;
        return true;
    }
    std::sort(vValue.begin(), vValue.end(), [](const ValuedCoin& a, const ValuedCoin& b) { return a.first > b.first; });
    std::vector<char> vfBest;
    Amount nBest;
    ApproximateBestSubset(vValue, nTotalLower, nTargetValue, vfBest, nBest);
    if (nBest != nTargetValue && nTotalLower >= nTargetValue + MIN_CHANGE)
        ApproximateBestSubset(vValue, nTotalLower, nTargetValue + MIN_CHANGE, vfBest, nBest);
    if (coinLowestLarger.second.first &&
        ((nBest != nTargetValue && nBest < nTargetValue + MIN_CHANGE) || coinLowestLarger.first <= nBest)) {
        setCoinsRet.insert(coinLowestLarger.second);
        nValueRet += coinLowestLarger.first;
    } else {
        for (size_t i = 0; i < vValue.size(); i++)
            if (vfBest[i]) {
                setCoinsRet.insert(vValue[i].second);
                nValueRet += vValue[i].first;
            }
    }
    return true;
}

bool CWallet::SelectCoins(const std::vector<COutput>& vAvailableCoins, Amount nTargetValue,
                          std::set<std::pair<const CWalletTx*, unsigned int>>& setCoinsRet, Amount& nValueRet,
                          const CCoinControl* coinControl) const {
    std::vector<COutput> vCoins(vAvailableCoins);
    if (coinControl && coinControl->HasSelected() && !coinControl->fAllowOtherInputs) {
        for (const COutput& o : vCoins) {
            if (!o.fSpendable) continue;
            nValueRet += o.tx->tx->vout[o.i].nValue;
            setCoinsRet.insert({o.tx, (unsigned)o.i});
        }
        return nValueRet >= nTargetValue;
    }
    // preset inputs chosen by coin control
    std::set<std::pair<const CWalletTx*, unsigned>> setPresetCoins;
    Amount nValueFromPresetInputs = 0;
    if (coinControl) {
        for (const COutPoint& o : coinControl->setSelected) {
            auto it = mapWallet.find(o.hash);
            if (it == mapWallet.end() || it->second.tx->vout.size() <= o.n) return false;
            nValueFromPresetInputs += it->second.tx->vout[o.n].nValue;
            setPresetCoins.insert({&it->second, o.n});
        }
    }
    for (auto it = vCoins.begin(); it != vCoins.end();) {
        if (setPresetCoins.count({it->tx, (unsigned)it->i})) it = vCoins.erase(it);
        else ++it;
    }
    // confirmed coins first, then unconfirmed change with ever longer mempool chains; beyond
    // the mempool's chain limits only without -walletrejectlongchains (reference wallet.cpp:2513-2540)
    const Amount target = nTargetValue - nValueFromPresetInputs;
    const uint64_t nMaxChainLength = (uint64_t)std::min(gArgs.GetArg("-limitancestorcount", (int64_t)DEFAULT_ANCESTOR_LIMIT),
                                                        gArgs.GetArg("-limitdescendantcount", (int64_t)DEFAULT_DESCENDANT_LIMIT));
    const bool fRejectLongChains = gArgs.GetBoolArg("-walletrejectlongchains", DEFAULT_WALLET_REJECT_LONG_CHAINS);
    const bool zc = gArgs.GetBoolArg("-spendzeroconfchange", DEFAULT_SPEND_ZEROCONF_CHANGE);
    bool res = target <= 0 || SelectCoinsMinConf(target, 1, 6, 0, vCoins, setCoinsRet, nValueRet) ||
               SelectCoinsMinConf(target, 1, 1, 0, vCoins, setCoinsRet, nValueRet) ||
               (zc && SelectCoinsMinConf(target, 0, 1, 2, vCoins, setCoinsRet, nValueRet)) ||
               (zc && SelectCoinsMinConf(target, 0, 1, std::min<uint64_t>(4, nMaxChainLength / 3), vCoins, setCoinsRet,
                                         nValueRet)) ||
               (zc && SelectCoinsMinConf(target, 0, 1, nMaxChainLength / 2, vCoins, setCoinsRet, nValueRet)) ||
               (zc && SelectCoinsMinConf(target, 0, 1, nMaxChainLength, vCoins, setCoinsRet, nValueRet)) ||
               (zc && !fRejectLongChains &&
                SelectCoinsMinConf(target, 0, 1, std::numeric_limits<uint64_t>::max(), vCoins, setCoinsRet, nValueRet));
    setCoinsRet.insert(setPresetCoins.begin(), setPresetCoins.end());
    nValueRet += nValueFromPresetInputs;
    return res;
}

Amount CWallet::GetMinimumFee(unsigned int nTxBytes, unsigned int nConfirmTarget) const {
    Amount nFee = payTxFee.GetFee(nTxBytes);
    if (nFee == 0) {
        CFeeRate rate;
        if (mempool && mempool->Estimator()) {
            int found = 0;
            rate = mempool->Estimator()->estimateSmartFee((int)nConfirmTarget, &found);
        }
        nFee = rate.GetFee(nTxBytes);
        if (nFee == 0)
            nFee = CFeeRate(gArgs.IsArgSet("-fallbackfee") ? [] {
                       int64_t n = DEFAULT_FALLBACK_FEE;
                       ParseMoney(gArgs.GetArg("-fallbackfee", ""), n);
                       return n;
                   }()
                                                           : DEFAULT_FALLBACK_FEE)
                       .GetFee(nTxBytes);
    }
    int64_t minTx = DEFAULT_TRANSACTION_MINFEE;
    if (gArgs.IsArgSet("-mintxfee")) ParseMoney(gArgs.GetArg("-mintxfee", ""), minTx);
    nFee = std::max(nFee, std::max(CFeeRate(minTx).GetFee(nTxBytes), minRelayTxFee.GetFee(nTxBytes)));
    int64_t maxTx = 10000000; // 0.1 BCP default -maxtxfee
    if (gArgs.IsArgSet("-maxtxfee")) ParseMoney(gArgs.GetArg("-maxtxfee", ""), maxTx);
    return std::min(nFee, (Amount)maxTx);
}

bool CWallet::CreateTransaction(const std::vector<CRecipient>& vecSend, CWalletTx& wtxNew, CReserveKey& reservekey,
                                Amount& nFeeRet, int& nChangePosInOut, std::string& strFailReason,
                                const CCoinControl* coinControl, bool sign) {
    Amount nValue = 0;
    const int nChangePosRequest = nChangePosInOut;
    unsigned int nSubtractFeeFromAmount = 0;
    for (const CRecipient& r : vecSend) {
        if (nValue < 0 || r.nAmount < 0) {
            strFailReason = "Transaction amounts must not be negative";
            return false;
        }
        nValue += r.nAmount;
        if (r.fSubtractFeeFromAmount) nSubtractFeeFromAmount++;
    }
    if (vecSend.empty()) {
        strFailReason = "Transaction must have at least one recipient";
        return false;
    }
    wtxNew.fTimeReceivedIsTxTime = true;
    wtxNew.pwallet = this;
    CMutableTransaction txNew;
    std::lock_guard<CCriticalSection> lm(chainstate->cs());
    WalletLock l(*this);
    // anti fee-sniping: lock to the current height, sometimes a bit earlier
    txNew.nLockTime = (uint32_t)chainstate->Height();
    if (GetRandInt(10) == 0) txNew.nLockTime = (uint32_t)std::max(0, (int)txNew.nLockTime - GetRandInt(100));
    std::vector<COutput> vAvailableCoins;
    AvailableCoins(vAvailableCoins, true, coinControl);
    nFeeRet = 0;
    const unsigned int confTarget = coinControl && coinControl->nConfirmTarget > 0 ? coinControl->nConfirmTarget
                                                                                   : nTxConfirmTarget;
    for (;;) {
        nChangePosInOut = nChangePosRequest;
        txNew.vin.clear();
        txNew.vout.clear();
        bool fFirst = true;
        const Amount nValueToSelect = nValue + (nSubtractFeeFromAmount == 0 ? nFeeRet : 0);
        for (const CRecipient& r : vecSend) {
            CTxOut txout(r.nAmount, r.scriptPubKey);
            if (r.fSubtractFeeFromAmount) {
                txout.nValue -= nFeeRet / nSubtractFeeFromAmount;
                if (fFirst) {
                    fFirst = false;
                    txout.nValue -= nFeeRet % nSubtractFeeFromAmount;
                }
            }
            if (IsDust(txout, dustRelayFee)) {
                if (r.fSubtractFeeFromAmount && nFeeRet > 0) {
                    strFailReason = txout.nValue < 0 ? "The transaction amount is too small to pay the fee"
                                                     : "The transaction amount is too small to send after the fee has been deducted";
                } else {
                    strFailReason = "Transaction amount too small";
                }
                return false;
            }
            txNew.vout.push_back(txout);
        }
        std::set<std::pair<const CWalletTx*, unsigned int>> setCoins;
        Amount nValueIn = 0;
        if (!SelectCoins(vAvailableCoins, nValueToSelect, setCoins, nValueIn, coinControl)) {
            strFailReason = "Insufficient funds";
            return false;
        }
        const Amount nChange = nValueIn - nValueToSelect;
        if (nChange > 0) {
            CScript scriptChange;
            if (coinControl && coinControl->destChange.IsValid()) {
                scriptChange = GetScriptForDestination(coinControl->destChange);
            } else {
                CPubKey vchPubKey;
                if (!reservekey.GetReservedKey(vchPubKey)) {
                    strFailReason = "Keypool ran out, please call keypoolrefill first";
                    return false;
                }
                scriptChange = GetScriptForDestination(vchPubKey.GetID());
            }
            CTxOut newTxOut(nChange, scriptChange);
            if (nSubtractFeeFromAmount > 0 && IsDust(newTxOut, dustRelayFee)) {
                // dust change goes to the first fee-paying recipient instead
                const Amount nDust = newTxOut.nValue;
                for (size_t i = 0; i < vecSend.size(); i++)
                    if (vecSend[i].fSubtractFeeFromAmount) {
                        txNew.vout[i].nValue += nDust;
                        break;
                    }
                newTxOut.nValue = 0;
            }
            if (IsDust(newTxOut, dustRelayFee)) {
                nChangePosInOut = -1;
                nFeeRet += newTxOut.nValue;
                reservekey.ReturnKey();
            } else {
                if (nChangePosInOut == -1) nChangePosInOut = GetRandInt((int)txNew.vout.size() + 1);
                else if ((size_t)nChangePosInOut > txNew.vout.size()) {
                    strFailReason = "Change index out of range";
                    return false;
                }
                txNew.vout.insert(txNew.vout.begin() + nChangePosInOut, newTxOut);
            }
        } else {
            reservekey.ReturnKey();
            nChangePosInOut = -1;
        }
        for (const auto& coin : setCoins)
            txNew.vin.push_back(CTxIn(COutPoint(coin.first->GetHash(), coin.second), CScript(),
                                      std::numeric_limits<uint32_t>::max() - 1));
        // sign (or dummy-sign to size the transaction)
        int nIn = 0;
        const CTransaction txConst(txNew);
        for (const auto& coin : setCoins) {
            const CScript& scriptPubKey = coin.first->tx->vout[coin.second].scriptPubKey;
            const Amount amount = coin.first->tx->vout[coin.second].nValue;
            SignatureData sigdata;
            const bool ok = sign ? ProduceSignature(TransactionSignatureCreator(this, &txConst, nIn, amount,
                                                                                SIGHASH_ALL | SIGHASH_FORKID),
                                                    scriptPubKey, sigdata)
                                 : ProduceSignature(DummySignatureCreator(this), scriptPubKey, sigdata);
            if (!ok) {
                strFailReason = "Signing transaction failed";
                return false;
            }
            UpdateTransaction(txNew, nIn, sigdata);
            nIn++;
        }
        const unsigned int nBytes = (unsigned int)GetSerializeSize(txNew);
        if (nBytes > MAX_STANDARD_TX_SIZE) {
            strFailReason = "Transaction too large";
            return false;
        }
        // a small, old-coin transaction may go free (-sendfreetransactions; reference wallet.cpp:2889-2899)
        if (fSendFreeTransactions && nBytes <= MAX_FREE_TRANSACTION_CREATE_SIZE && mempool) {
            double dPriority = 0;
            for (const auto& coin : setCoins)
                dPriority += (double)coin.first->tx->vout[coin.second].nValue * coin.first->GetDepthInMainChain();
            unsigned nModSize = nBytes;
            for (const CTxIn& in : txNew.vin) {
                const unsigned offset = 41U + std::min(110U, (unsigned)in.scriptSig.size());
                if (nModSize > offset) nModSize -= offset;
            }
            dPriority = nModSize ? dPriority / nModSize : 0;
            int found = 0;
            // a mempool that is full enough to charge a minimum fee takes nothing free
            // (reference txmempool.cpp estimateSmartPriority)
            const size_t maxmempool = (size_t)gArgs.GetArg("-maxmempool", (int64_t)DEFAULT_MAX_MEMPOOL_SIZE) * 1000000;
            const double dPriorityNeeded = mempool->GetMinFee(maxmempool).GetFeePerK() > 0 || !mempool->Estimator()
                                               ? 1e16
                                               : mempool->Estimator()->estimateSmartPriority((int)confTarget, &found);
            if (dPriority >= dPriorityNeeded && AllowFree(dPriority)) {
                wtxNew.tx = MakeTransactionRef(std::move(txNew));
                break;
            }
        }
        Amount nFeeNeeded = GetMinimumFee(nBytes, confTarget);
        if (coinControl && coinControl->fOverrideFeeRate) nFeeNeeded = coinControl->nFeeRate.GetFee(nBytes);
        if (nFeeNeeded < minRelayTxFee.GetFee(nBytes)) {
            strFailReason = "Transaction too large for fee policy";
            return false;
        }
        if (nFeeRet >= nFeeNeeded) {
            // overpaid because of a dropped change output is fine; otherwise done
            wtxNew.tx = MakeTransactionRef(std::move(txNew));
            break;
        }
        nFeeRet = nFeeNeeded;
    }
    if (gArgs.GetBoolArg("-walletrejectlongchains", DEFAULT_WALLET_REJECT_LONG_CHAINS) && mempool) {
        // the transaction must pass the mempool's chain limits (reference wallet.cpp:3000-3025)
        CTxMemPoolEntry entry(wtxNew.tx, 0, 0, 0.0, 0, 0, false, 0, LockPoints());
        CTxMemPool::setEntries setAncestors;
        std::string errString;
        std::lock_guard<CCriticalSection> lmp(mempool->cs);
        if (!mempool->CalculateMemPoolAncestors(
                entry, setAncestors, (uint64_t)gArgs.GetArg("-limitancestorcount", (int64_t)DEFAULT_ANCESTOR_LIMIT),
                (uint64_t)gArgs.GetArg("-limitancestorsize", (int64_t)DEFAULT_ANCESTOR_SIZE_LIMIT) * 1000,
                (uint64_t)gArgs.GetArg("-limitdescendantcount", (int64_t)DEFAULT_DESCENDANT_LIMIT),
                (uint64_t)gArgs.GetArg("-limitdescendantsize", (int64_t)DEFAULT_DESCENDANT_SIZE_LIMIT) * 1000, errString)) {
            strFailReason = "Transaction has too long of a mempool chain";
            return false;
        }
    }
    return true;
}

bool CWallet::CommitTransaction(CWalletTx& wtxNew, CReserveKey& reservekey, CValidationState& state) {
    std::lock_guard<CCriticalSection> lm(chainstate->cs());
    WalletLock l(*this);
    LogPrintf("CommitTransaction:\n%s", wtxNew.tx->ToString().c_str());
    reservekey.KeepKey();
    wtxNew.fFromMe = true;
    AddToWallet(wtxNew);
    CWalletTx& stored = mapWallet.at(wtxNew.GetHash());
    if (fBroadcastTransactions) {
        if (!chainstate->AcceptToMemoryPool(state, stored.tx, false, nullptr, false, 0)) {
            LogPrintf("CommitTransaction(): Transaction cannot be broadcast immediately, %s\n",
                      FormatStateMessage(state).c_str());
            return false;
        }
        stored.RelayWalletTransaction();
    }
    return true;
}

bool CWallet::FundTransaction(CMutableTransaction& tx, Amount& nFeeRet, bool overrideEstimatedFeeRate,
                              const CFeeRate& specificFeeRate, int& nChangePosInOut, std::string& strFailReason,
                              bool includeWatching, bool lockUnspents, const std::set<int>& setSubtractFeeFromOutputs,
                              bool keepReserveKey, const CTxDestination& destChange) {
    std::vector<CRecipient> vecSend;
    for (size_t i = 0; i < tx.vout.size(); i++)
        vecSend.push_back({tx.vout[i].scriptPubKey, tx.vout[i].nValue, setSubtractFeeFromOutputs.count((int)i) > 0});
    CCoinControl cc;
    cc.destChange = destChange;
    cc.fAllowOtherInputs = true;
    cc.fAllowWatchOnly = includeWatching;
    cc.fOverrideFeeRate = overrideEstimatedFeeRate;
    cc.nFeeRate = specificFeeRate;
    for (const CTxIn& in : tx.vin) cc.setSelected.insert(in.prevout);
    CReserveKey reservekey(this);
    CWalletTx wtx;
    if (!CreateTransaction(vecSend, wtx, reservekey, nFeeRet, nChangePosInOut, strFailReason, &cc, false)) return false;
    if (nChangePosInOut != -1) tx.vout.insert(tx.vout.begin() + nChangePosInOut, wtx.tx->vout[nChangePosInOut]);
    // copy output amounts (fee subtraction may have changed them)
    for (size_t i = 0; i < tx.vout.size(); i++) {
        const size_t j = (nChangePosInOut != -1 && (int)i >= nChangePosInOut) ? i : i;
        tx.vout[i].nValue = wtx.tx->vout[j].nValue;
    }
    // add new inputs, keep existing ones (and their scriptSigs)
    for (const CTxIn& in : wtx.tx->vin) {
        bool have = false;
        for (const CTxIn& e : tx.vin)
            if (e.prevout == in.prevout) have = true;
        if (!have) {
            tx.vin.push_back(CTxIn(in.prevout, CScript(), in.nSequence));
            if (lockUnspents) LockCoin(in.prevout);
        }
    }
    if (keepReserveKey) reservekey.KeepKey();
    return true;
}

void CWallet::LockCoin(const COutPoint& o) {
    WalletLock l(*this);
    setLockedCoins.insert(o);
}
void CWallet::UnlockCoin(const COutPoint& o) {
    WalletLock l(*this);
    setLockedCoins.erase(o);
}
void CWallet::UnlockAllCoins() {
    WalletLock l(*this);
    setLockedCoins.clear();
}
bool CWallet::IsLockedCoin(const uint256& hash, unsigned int n) const {
    WalletLock l(*this);
    return setLockedCoins.count(COutPoint(hash, n)) > 0;
}
std::vector<COutPoint> CWallet::ListLockedCoins() const {
    WalletLock l(*this);
    return std::vector<COutPoint>(setLockedCoins.begin(), setLockedCoins.end());
}

bool CWallet::SetAddressBook(const CTxDestination& address, const std::string& strName, const std::string& purpose) {
    WalletLock l(*this);
    CAddressBookData& d = mapAddressBook[address];
    d.name = strName;
    if (!purpose.empty()) d.purpose = purpose;
    KVBatch b;
    if (!purpose.empty()) b.Write(K("purpose", DestKey{address}), purpose);
    b.Write(K("name", DestKey{address}), strName);
    return db->WriteBatch(b, true);
}

bool CWallet::DelAddressBook(const CTxDestination& address) {
    WalletLock l(*this);
    KVBatch b;
    for (const auto& kv : mapAddressBook[address].destdata) b.Erase(K("destdata", std::make_pair(DestKey{address}, kv.first)));
    mapAddressBook.erase(address);
    b.Erase(K("purpose", DestKey{address}));
    b.Erase(K("name", DestKey{address}));
    return db->WriteBatch(b, true);
}

bool CWallet::AddDestData(const CTxDestination& dest, const std::string& key, const std::string& value) {
    if (!dest.IsValid()) return false;
    WalletLock l(*this);
    mapAddressBook[dest].destdata[key] = value;
    return db->Write(K("destdata", std::make_pair(DestKey{dest}, key)), value, true);
}

bool CWallet::EraseDestData(const CTxDestination& dest, const std::string& key) {
    WalletLock l(*this);
    auto it = mapAddressBook.find(dest);
    if (it == mapAddressBook.end() || !it->second.destdata.erase(key)) return false;
    return db->Erase(K("destdata", std::make_pair(DestKey{dest}, key)), true);
}

bool CWallet::GetDestData(const CTxDestination& dest, const std::string& key, std::string* value) const {
    WalletLock l(*this);
    auto it = mapAddressBook.find(dest);
    if (it == mapAddressBook.end()) return false;
    auto d = it->second.destdata.find(key);
    if (d == it->second.destdata.end()) return false;
    if (value) *value = d->second;
    return true;
}

bool CWallet::GetAccountPubkey(CPubKey& pubKey, const std::string& strAccount, bool bForceNew) {
    WalletLock l(*this);
    CPubKey cur;
    const bool have = db->Read(K("acc", strAccount), cur);
    bool keyUsed = false;
    if (have && cur.IsValid()) {
        const CScript script = GetScriptForDestination(cur.GetID());
        for (const auto& kv : mapWallet) {
            for (const CTxOut& o : kv.second.tx->vout)
                if (o.scriptPubKey == script) keyUsed = true;
            if (keyUsed) break;
        }
    }
    if (!have || !cur.IsValid() || bForceNew || keyUsed) {
        if (!GetKeyFromPool(cur)) return false;
        SetAddressBook(cur.GetID(), strAccount, "receive");
        db->Write(K("acc", strAccount), cur, true);
    }
    pubKey = cur;
    return true;
}

} // namespace bcp
