// Wallet.
// Parity: reference src/wallet/wallet.{h,cpp} (CWallet: key pool, HD chain m/0'/0'/k',
// encryption, transaction tracking via validation callbacks, IsMine, balances,
// AvailableCoins/knapsack coin selection, CreateTransaction with SIGHASH_ALL|FORKID
// signing and fee computation from -paytxfee/-fallbackfee/-mintxfee/estimates,
// CommitTransaction + relay, rescans, abandon, accounts/address book, locked coins,
// resend), src/wallet/walletdb.{h,cpp} (record types), src/wallet/rpcwallet.cpp and
// rpcdump.cpp (RPC surface, registered in wallet/rpcwallet.cpp).
//
// Storage: wallet records live in a KVStore directory (<datadir>/<-wallet>) using the
// reference's record names ("key", "ckey", "mkey", "tx", "name", "pool", "hdchain", ...)
// instead of a Berkeley DB file; backupwallet writes a compacted copy.
#pragma once
#include "consensus/chain.h"
#include "node/kvstore.h"
#include "node/signals.h"
#include "primitives/amount.h"
#include "primitives/transaction.h"
#include "script/standard.h"
#include "wallet/crypter.h"

#include <atomic>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

namespace bcp {

class Chainstate;
class CTxMemPool;
class CWallet;

static const unsigned int DEFAULT_KEYPOOL_SIZE = 100;
static const Amount DEFAULT_TRANSACTION_FEE = 0;
static const Amount DEFAULT_FALLBACK_FEE = 20000;
static const Amount DEFAULT_TRANSACTION_MINFEE = 1000;
static const Amount MIN_CHANGE = 1000000; // CENT
static const Amount MIN_FINAL_CHANGE = MIN_CHANGE / 2;
static const unsigned int DEFAULT_TX_CONFIRM_TARGET = 6;
static const bool DEFAULT_SPEND_ZEROCONF_CHANGE = true;
static const bool DEFAULT_SEND_FREE_TRANSACTIONS = false;
static const bool DEFAULT_WALLET_REJECT_LONG_CHAINS = false;
static const unsigned int MAX_FREE_TRANSACTION_CREATE_SIZE = 1000;
static const bool DEFAULT_FLUSHWALLET = true;
static const bool DEFAULT_WALLETBROADCAST = true;
// wallet format versions (reference wallet.h WalletFeature): a store records the lowest client
// version that can open it ("minversion")
static const int WALLET_FEATURE_BASE = 10500;
static const int WALLET_FEATURE_WALLETCRYPT = 40000;
static const int WALLET_FEATURE_COMPRPUBKEY = 60000;
static const int WALLET_FEATURE_HD = 130000;
static const int WALLET_FEATURE_LATEST = WALLET_FEATURE_COMPRPUBKEY; // HD is optional

enum isminetype : uint8_t {
    ISMINE_NO = 0,
    ISMINE_WATCH_UNSOLVABLE = 1,
    ISMINE_WATCH_SOLVABLE = 2,
    ISMINE_WATCH_ONLY = ISMINE_WATCH_SOLVABLE | ISMINE_WATCH_UNSOLVABLE,
    ISMINE_SPENDABLE = 4,
    ISMINE_ALL = ISMINE_WATCH_ONLY | ISMINE_SPENDABLE
};
typedef uint8_t isminefilter;

isminetype IsMine(const CKeyStore& ks, const CScript& script);
isminetype IsMine(const CKeyStore& ks, const CTxDestination& dest);

struct CKeyMetadata {
    int32_t nVersion = 10;
    int64_t nCreateTime = 0;
    std::string hdKeypath;
    CKeyID hdMasterKeyID;
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, nVersion);
        ::bcp::Serialize(s, nCreateTime);
        ::bcp::Serialize(s, hdKeypath);
        ::bcp::Serialize(s, hdMasterKeyID);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, nVersion);
        ::bcp::Unserialize(s, nCreateTime);
        ::bcp::Unserialize(s, hdKeypath);
        ::bcp::Unserialize(s, hdMasterKeyID);
    }
};

struct CHDChain {
    int32_t nVersion = 1;
    uint32_t nExternalChainCounter = 0;
    CKeyID masterKeyID;
    bool IsNull() const { return masterKeyID.IsNull(); }
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, nVersion);
        ::bcp::Serialize(s, nExternalChainCounter);
        ::bcp::Serialize(s, masterKeyID);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, nVersion);
        ::bcp::Unserialize(s, nExternalChainCounter);
        ::bcp::Unserialize(s, masterKeyID);
    }
};

struct CKeyPool {
    int64_t nTime = 0;
    CPubKey vchPubKey;
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, nTime);
        ::bcp::Serialize(s, vchPubKey);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, nTime);
        ::bcp::Unserialize(s, vchPubKey);
    }
};

struct CAddressBookData {
    std::string name;
    std::string purpose = "unknown";
    std::map<std::string, std::string> destdata;
};

// Internal transfer between accounts (reference CAccountingEntry).
struct CAccountingEntry {
    std::string strAccount;
    Amount nCreditDebit = 0;
    int64_t nTime = 0;
    std::string strOtherAccount;
    std::string strComment;
    int64_t nOrderPos = -1;
    uint64_t nEntryNo = 0;
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, strAccount);
        ::bcp::Serialize(s, nCreditDebit);
        ::bcp::Serialize(s, nTime);
        ::bcp::Serialize(s, strOtherAccount);
        ::bcp::Serialize(s, strComment);
        ::bcp::Serialize(s, nOrderPos);
        ::bcp::Serialize(s, nEntryNo);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, strAccount);
        ::bcp::Unserialize(s, nCreditDebit);
        ::bcp::Unserialize(s, nTime);
        ::bcp::Unserialize(s, strOtherAccount);
        ::bcp::Unserialize(s, strComment);
        ::bcp::Unserialize(s, nOrderPos);
        ::bcp::Unserialize(s, nEntryNo);
    }
};

struct COutputEntry {
    CTxDestination destination;
    Amount amount;
    int vout;
};

class CWalletTx {
public:
    CWalletTx() {}
    CWalletTx(const CWallet* w, CTransactionRef t) : pwallet(w), tx(std::move(t)) {}
    static const uint256 ABANDON_HASH;

    const CWallet* pwallet = nullptr;
    CTransactionRef tx;
    uint256 hashBlock;           // null: unconfirmed; ABANDON_HASH: abandoned
    int nIndex = -1;             // position in block; -1 with hashBlock set = conflicted by that block
    std::map<std::string, std::string> mapValue;
    std::vector<std::pair<std::string, std::string>> vOrderForm;
    bool fTimeReceivedIsTxTime = false;
    uint32_t nTimeReceived = 0;
    uint32_t nTimeSmart = 0;
    bool fFromMe = false;
    std::string strFromAccount;
    int64_t nOrderPos = -1;

    const uint256& GetHash() const { return tx->GetHash(); }
    bool IsCoinBase() const { return tx->IsCoinBase(); }
    bool IsAbandoned() const { return hashBlock == ABANDON_HASH; }
    void SetAbandoned() {
        hashBlock = ABANDON_HASH;
        nIndex = -1;
    }
    bool IsUnconfirmed() const { return hashBlock.IsNull() || IsAbandoned(); }
    int GetDepthInMainChain(const CBlockIndex** ppindex = nullptr) const;
    int GetBlocksToMaturity() const;
    bool IsInMainChain() const { return GetDepthInMainChain() > 0; }
    bool InMempool() const;
    bool IsTrusted() const;
    int64_t GetTxTime() const { return nTimeSmart ? nTimeSmart : nTimeReceived; }
    Amount GetDebit(const isminefilter& filter) const;
    Amount GetCredit(const isminefilter& filter) const;
    Amount GetImmatureCredit(bool fUseCache = true) const;
    Amount GetAvailableCredit(bool fUseCache = true) const;
    Amount GetImmatureWatchOnlyCredit() const;
    Amount GetAvailableWatchOnlyCredit() const;
    Amount GetChange() const;
    bool IsFromMe(const isminefilter& filter) const { return GetDebit(filter) > 0; }
    bool IsEquivalentTo(const CWalletTx& o) const;
    void GetAmounts(std::list<COutputEntry>& listReceived, std::list<COutputEntry>& listSent, Amount& nFee,
                    std::string& strSentAccount, const isminefilter& filter) const;
    std::set<uint256> GetConflicts() const;
    bool RelayWalletTransaction();

    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, *tx);
        ::bcp::Serialize(s, hashBlock);
        ::bcp::Serialize(s, nIndex);
        std::map<std::string, std::string> mv = mapValue;
        mv["fromaccount"] = strFromAccount;
        mv["n"] = std::to_string(nOrderPos);
        if (nTimeSmart) mv["timesmart"] = std::to_string(nTimeSmart);
        ::bcp::Serialize(s, mv);
        ::bcp::Serialize(s, vOrderForm);
        const uint8_t flags = (fTimeReceivedIsTxTime ? 1 : 0) | (fFromMe ? 2 : 0);
        ::bcp::Serialize(s, nTimeReceived);
        ::bcp::Serialize(s, flags);
    }
    template <typename S> void Unserialize(S& s) {
        CMutableTransaction mtx;
        ::bcp::Unserialize(s, mtx);
        tx = MakeTransactionRef(std::move(mtx));
        ::bcp::Unserialize(s, hashBlock);
        ::bcp::Unserialize(s, nIndex);
        ::bcp::Unserialize(s, mapValue);
        ::bcp::Unserialize(s, vOrderForm);
        uint8_t flags = 0;
        ::bcp::Unserialize(s, nTimeReceived);
        ::bcp::Unserialize(s, flags);
        fTimeReceivedIsTxTime = flags & 1;
        fFromMe = (flags & 2) != 0;
        strFromAccount = mapValue["fromaccount"];
        nOrderPos = mapValue.count("n") ? std::stoll(mapValue["n"]) : -1;
        nTimeSmart = mapValue.count("timesmart") ? (uint32_t)std::stoul(mapValue["timesmart"]) : 0;
        mapValue.erase("fromaccount");
        mapValue.erase("n");
        mapValue.erase("timesmart");
    }
};

struct COutput {
    const CWalletTx* tx;
    int i;
    int nDepth;
    bool fSpendable;
    bool fSolvable;
};

struct CRecipient {
    CScript scriptPubKey;
    Amount nAmount;
    bool fSubtractFeeFromAmount;
};

// Options for fundrawtransaction / coin selection (reference src/wallet/coincontrol.h).
struct CCoinControl {
    CTxDestination destChange;
    bool fAllowOtherInputs = false;
    bool fAllowWatchOnly = false;
    bool fOverrideFeeRate = false;
    CFeeRate nFeeRate;
    int nConfirmTarget = 0;
    std::set<COutPoint> setSelected;
    bool HasSelected() const { return !setSelected.empty(); }
    bool IsSelected(const COutPoint& o) const { return setSelected.count(o) > 0; }
};

class CReserveKey {
public:
    explicit CReserveKey(CWallet* w) : pwallet(w) {}
    ~CReserveKey() { ReturnKey(); }
    bool GetReservedKey(CPubKey& pubkey);
    void KeepKey();
    void ReturnKey();

private:
    CWallet* pwallet;
    int64_t nIndex = -1;
    CPubKey vchPubKey;
};

class CWallet : public CCryptoKeyStore, public CValidationInterface {
public:
    CWallet(const std::string& name, const std::string& path, bool memoryOnly = false);
    ~CWallet();

    // ---- lifecycle
    bool Load(std::string& err, bool& firstRun); // read every record
    void Attach(Chainstate* cs, CTxMemPool* pool) {
        chainstate = cs;
        mempool = pool;
    }
    bool ScanForWalletTransactions(const CBlockIndex* pindexStart, bool fUpdate, int* pnFound = nullptr);
    void ReacceptWalletTransactions();
    void Flush();
    bool BackupWallet(const std::string& dest);
    const std::string& GetName() const { return strWalletName; }

    // ---- keys
    CPubKey GenerateNewKey();
    bool AddKeyPubKey(const CKey& key, const CPubKey& pubkey) override;
    bool LoadKey(const CKey& key, const CPubKey& pubkey) { return CCryptoKeyStore::AddKeyPubKey(key, pubkey); }
    bool AddCryptedKey(const CPubKey& pubkey, const std::vector<unsigned char>& crypted) override;
    bool AddCScript(const CScript& redeemScript) override;
    bool AddWatchOnly(const CScript& dest) override;
    bool AddWatchOnly(const CScript& dest, int64_t nCreateTime);
    bool RemoveWatchOnly(const CScript& dest) override;
    bool HaveWatchOnly(const CScript& dest) const override { return CBasicKeyStore::HaveWatchOnly(dest); }
    bool HaveWatchOnly() const override { return CBasicKeyStore::HaveWatchOnly(); }
    std::map<CKeyID, CKeyMetadata> mapKeyMetadata;
    std::map<CScriptID, CKeyMetadata> mapScriptMetadata;
    int64_t nTimeFirstKey = 0;
    void UpdateTimeFirstKey(int64_t nCreateTime);

    // HD
    bool IsHDEnabled() const { return !hdChain.IsNull(); }
    CPubKey GenerateNewHDMasterKey();
    bool SetHDMasterKey(const CPubKey& key);
    const CHDChain& GetHDChain() const { return hdChain; }

    // key pool
    bool NewKeyPool();
    bool TopUpKeyPool(unsigned int kpSize = 0);
    void ReserveKeyFromKeyPool(int64_t& nIndex, CKeyPool& keypool);
    void KeepKey(int64_t nIndex);
    void ReturnKey(int64_t nIndex);
    bool GetKeyFromPool(CPubKey& key);
    int64_t GetOldestKeyPoolTime();
    size_t KeypoolCountExternalKeys() const { return setKeyPool.size(); }

    // encryption
    bool EncryptWallet(const std::string& passphrase);
    bool Unlock(const std::string& passphrase);
    bool ChangeWalletPassphrase(const std::string& oldPass, const std::string& newPass);
    int64_t nRelockTime = 0;

    // ---- transactions
    std::map<uint256, CWalletTx> mapWallet;
    std::list<CAccountingEntry> laccentries;
    typedef std::pair<CWalletTx*, CAccountingEntry*> TxPair;
    std::multimap<int64_t, TxPair> wtxOrdered;
    int64_t nOrderPosNext = 0;
    int64_t IncOrderPosNext();
    const CWalletTx* GetWalletTx(const uint256& hash) const;
    bool AddToWallet(const CWalletTx& wtxIn, bool fFlushOnClose = true);
    bool AddToWalletIfInvolvingMe(const CTransactionRef& tx, const CBlockIndex* pIndex, int posInBlock, bool fUpdate);
    bool AbandonTransaction(const uint256& hashTx);
    bool MarkConflicted(const uint256& hashBlock, const uint256& hashTx);
    void SyncTransaction(const CTransactionRef& tx, const CBlockIndex* pindex = nullptr, int posInBlock = 0);
    std::vector<uint256> ResendWalletTransactionsBefore(int64_t nTime);
    bool AddAccountingEntry(const CAccountingEntry& entry);
    // Gives unordered transactions and account-"" accounting entries (nOrderPos -1: wallets
    // from before ordering existed) positions by receive time, shifting the ordered ones past
    // them, and writes back what moved (reference CWallet::ReorderTransactions, run by
    // LoadWallet when any record is unordered).
    bool ReorderTransactions();

    // ---- ownership / amounts
    isminetype IsMine(const CTxIn& txin) const;
    isminetype IsMine(const CTxOut& txout) const;
    bool IsMine(const CTransaction& tx) const;
    bool IsFromMe(const CTransaction& tx) const;
    Amount GetDebit(const CTxIn& txin, const isminefilter& filter) const;
    Amount GetDebit(const CTransaction& tx, const isminefilter& filter) const;
    Amount GetCredit(const CTxOut& txout, const isminefilter& filter) const;
    Amount GetCredit(const CTransaction& tx, const isminefilter& filter) const;
    bool IsChange(const CTxOut& txout) const;
    Amount GetChange(const CTxOut& txout) const;
    bool IsSpent(const uint256& hash, unsigned int n) const;
    Amount GetBalance() const;
    Amount GetUnconfirmedBalance() const;
    Amount GetImmatureBalance() const;
    Amount GetWatchOnlyBalance() const;
    Amount GetUnconfirmedWatchOnlyBalance() const;
    Amount GetImmatureWatchOnlyBalance() const;
    Amount GetAccountBalance(const std::string& strAccount, int nMinDepth, const isminefilter& filter);
    std::map<CTxDestination, Amount> GetAddressBalances();
    std::set<std::set<CTxDestination>> GetAddressGroupings();
    std::set<CTxDestination> GetAccountAddresses(const std::string& strAccount) const;

    // ---- spending
    void AvailableCoins(std::vector<COutput>& vCoins, bool fOnlyConfirmed = true, const CCoinControl* coinControl = nullptr,
                        bool fIncludeZeroValue = false) const;
    bool SelectCoinsMinConf(Amount nTargetValue, int nConfMine, int nConfTheirs, uint64_t nMaxAncestors, std::vector<COutput> vCoins,
                            std::set<std::pair<const CWalletTx*, unsigned int>>& setCoinsRet, Amount& nValueRet) const;
    bool SelectCoins(const std::vector<COutput>& vAvailableCoins, Amount nTargetValue,
                     std::set<std::pair<const CWalletTx*, unsigned int>>& setCoinsRet, Amount& nValueRet,
                     const CCoinControl* coinControl = nullptr) const;
    bool CreateTransaction(const std::vector<CRecipient>& vecSend, CWalletTx& wtxNew, CReserveKey& reservekey,
                           Amount& nFeeRet, int& nChangePosInOut, std::string& strFailReason,
                           const CCoinControl* coinControl = nullptr, bool sign = true);
    bool CommitTransaction(CWalletTx& wtxNew, CReserveKey& reservekey, CValidationState& state);
    bool FundTransaction(CMutableTransaction& tx, Amount& nFeeRet, bool overrideEstimatedFeeRate,
                         const CFeeRate& specificFeeRate, int& nChangePosInOut, std::string& strFailReason,
                         bool includeWatching, bool lockUnspents, const std::set<int>& setSubtractFeeFromOutputs,
                         bool keepReserveKey, const CTxDestination& destChange);
    Amount GetMinimumFee(unsigned int nTxBytes, unsigned int nConfirmTarget) const;
    void LockCoin(const COutPoint& o);
    void UnlockCoin(const COutPoint& o);
    void UnlockAllCoins();
    bool IsLockedCoin(const uint256& hash, unsigned int n) const;
    std::vector<COutPoint> ListLockedCoins() const;

    // ---- address book
    std::map<CTxDestination, CAddressBookData> mapAddressBook;
    bool SetAddressBook(const CTxDestination& address, const std::string& strName, const std::string& purpose);
    bool DelAddressBook(const CTxDestination& address);
    // Per-destination key/value data (reference wallet.cpp AddDestData/EraseDestData/GetDestData:
    // e.g. payment requests "rr<id>" and "used" markers), stored with the address book.
    bool AddDestData(const CTxDestination& dest, const std::string& key, const std::string& value);
    bool EraseDestData(const CTxDestination& dest, const std::string& key);
    bool GetDestData(const CTxDestination& dest, const std::string& key, std::string* value) const;
    bool GetAccountPubkey(CPubKey& pubKey, const std::string& strAccount, bool bForceNew = false);

    // ---- validation callbacks
    void TransactionAddedToMempool(const CTransactionRef& tx) override;
    void BlockConnected(const std::shared_ptr<const CBlock>& block, const CBlockIndex* pindex,
                        const std::vector<CTransactionRef>& txnConflicted) override;
    void BlockDisconnected(const std::shared_ptr<const CBlock>& block) override;
    void SetBestChain(const CBlockLocator& loc) override;
    void ResendWalletTransactions(int64_t nBestBlockTime) override;

    mutable CCriticalSection cs_wallet{"cs_wallet"};
    Chainstate* chainstate = nullptr;
    CTxMemPool* mempool = nullptr;
    CFeeRate payTxFee{DEFAULT_TRANSACTION_FEE};
    unsigned int nTxConfirmTarget = DEFAULT_TX_CONFIRM_TARGET;
    bool fSendFreeTransactions = DEFAULT_SEND_FREE_TRANSACTIONS; // -sendfreetransactions
    int nWalletVersion = 0, nWalletMaxVersion = 0;                 // "minversion" record, -upgradewallet cap
    void SetMinVersion(int v);
    void FlushIfDirty(); // -flushwallet: fsync the store if anything was written since the last call
    int GetVersion() const { return nWalletVersion; }
    bool fBroadcastTransactions = DEFAULT_WALLETBROADCAST;
    CPubKey vchDefaultKey;
    KVStore& DB() { return *db; }

private:
    bool WriteKeyRecords(const CPubKey& pub, const CKey* key, const std::vector<unsigned char>* crypted);
    void AddToSpends(const uint256& wtxid);
    void AddToSpends(const COutPoint& outpoint, const uint256& wtxid);
    void SyncMetaData(const COutPoint& outpoint);
    CPubKey DeriveNewChildKey(CKeyMetadata& metadata, CKey& secret);

    std::string strWalletName;
    std::string strWalletPath; // the store's directory (BackupWallet refuses to write onto it)
    uint64_t nLastFlushBytes = 0;
    std::unique_ptr<KVStore> db;
    std::map<unsigned int, CMasterKey> mapMasterKeys;
    unsigned int nMasterKeyMaxID = 0;
    CHDChain hdChain;
    std::set<int64_t> setKeyPool;
    std::set<COutPoint> setLockedCoins;
    std::multimap<COutPoint, uint256> mapTxSpends;
    int64_t nNextResend = 0;
    int64_t nLastResend = 0;
    uint64_t nAccountingEntryNumber = 0;
    friend class CWalletTx;
};

// Lock order cs_main -> cs_wallet (reference LOCK2(cs_main, pwallet->cs_wallet)): wallet
// code reads chain depth under cs_wallet, so every wallet critical section takes cs_main
// first when the wallet is attached to a chainstate.
class WalletLock {
public:
    explicit WalletLock(const CWallet& w);

private:
    std::unique_lock<CCriticalSection> m, l;
};

CWallet* GetWallet();
std::vector<CWallet*> GetWallets();

} // namespace bcp
