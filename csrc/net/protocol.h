// P2P wire protocol: message header, command names, inventory vectors.
// Parity: reference src/protocol.{h,cpp} (CMessageHeader 4+12+4+4 bytes with
// SHA256d checksum prefix, NetMsgType command strings, GetInv types MSG_TX/MSG_BLOCK/
// MSG_FILTERED_BLOCK/MSG_CMPCT_BLOCK), src/version.h protocol versions, and the P2P
// limits of src/net.h:51-83 / src/validation.h:93-164 / src/net_processing.h:16-20.
#pragma once
#include "net/netaddress.h"
#include "primitives/uint256.h"

#include <array>
#include <string>
#include <vector>

namespace bcp {

static const int GETHEADERS_VERSION = 31800;
static const int MEMPOOL_GD_VERSION = 60002;
static const int INVALID_CB_NO_BAN_VERSION = 70015;

// net.h limits
static const int PING_INTERVAL = 2 * 60;
static const int TIMEOUT_INTERVAL = 20 * 60;
static const int FEELER_INTERVAL = 120;
static const unsigned int MAX_INV_SZ = 50000;
static const unsigned int MAX_ADDR_TO_SEND = 1000;
static const unsigned int MAX_PROTOCOL_MESSAGE_LENGTH = 32 * 1000 * 1000;
static const unsigned int MAX_SUBVERSION_LENGTH = 256;
static const int MAX_OUTBOUND_CONNECTIONS = 8;
static const int MAX_ADDNODE_CONNECTIONS = 8;
static const unsigned int DEFAULT_MAX_PEER_CONNECTIONS = 125;
static const int64_t DEFAULT_BANSCORE_THRESHOLD = 100;
static const int64_t DEFAULT_MISBEHAVING_BANTIME = 60 * 60 * 24;
static const int DUMP_ADDRESSES_INTERVAL = 900;
// validation.h / net_processing.h limits
static const int MAX_BLOCKS_IN_TRANSIT_PER_PEER = 16;
static const unsigned int BLOCK_STALLING_TIMEOUT = 2;
static const unsigned int MAX_HEADERS_RESULTS = 2000;
static const int MAX_CMPCTBLOCK_DEPTH = 5;
static const int MAX_BLOCKTXN_DEPTH = 10;
static const unsigned int BLOCK_DOWNLOAD_WINDOW = 1024;
static const int MAX_UNCONNECTING_HEADERS = 10;
static const unsigned int DEFAULT_MAX_ORPHAN_TRANSACTIONS = 100;
static const int64_t ORPHAN_TX_EXPIRE_TIME = 20 * 60;
static const int64_t ORPHAN_TX_EXPIRE_INTERVAL = 5 * 60;
static const unsigned int MAX_BLOCKS_TO_ANNOUNCE = 8;
static const unsigned int INVENTORY_BROADCAST_INTERVAL = 5;
static const unsigned int INVENTORY_BROADCAST_MAX = 7 * INVENTORY_BROADCAST_INTERVAL;
static const int64_t BLOCK_DOWNLOAD_TIMEOUT_BASE = 1000000; // fraction of block interval (1e6 = 1x)
static const int64_t BLOCK_DOWNLOAD_TIMEOUT_PER_PEER = 500000;
static const unsigned int MAX_GETBLOCKS_RESULTS = 500;
static const unsigned int MAX_REJECT_MESSAGE_LENGTH = 111;
static const unsigned int REJECT_INTERNAL = 0x100; // never sent on the wire

namespace NetMsgType {
extern const char* VERSION;
extern const char* VERACK;
extern const char* ADDR;
extern const char* INV;
extern const char* GETDATA;
extern const char* MERKLEBLOCK;
extern const char* GETBLOCKS;
extern const char* GETHEADERS;
extern const char* TX;
extern const char* HEADERS;
extern const char* BLOCK;
extern const char* GETADDR;
extern const char* MEMPOOL;
extern const char* PING;
extern const char* PONG;
extern const char* NOTFOUND;
extern const char* FILTERLOAD;
extern const char* FILTERADD;
extern const char* FILTERCLEAR;
extern const char* REJECT;
extern const char* SENDHEADERS;
extern const char* FEEFILTER;
extern const char* SENDCMPCT;
extern const char* CMPCTBLOCK;
extern const char* GETBLOCKTXN;
extern const char* BLOCKTXN;
} // namespace NetMsgType
const std::vector<std::string>& GetAllNetMessageTypes();

class CMessageHeader {
public:
    static constexpr size_t MESSAGE_START_SIZE = 4, COMMAND_SIZE = 12, CHECKSUM_SIZE = 4;
    static constexpr size_t HEADER_SIZE = MESSAGE_START_SIZE + COMMAND_SIZE + 4 + CHECKSUM_SIZE;
    typedef std::array<unsigned char, MESSAGE_START_SIZE> MessageStartChars;

    CMessageHeader() { magic.fill(0); command.fill(0); checksum.fill(0); }
    CMessageHeader(const unsigned char* start, const char* cmd, uint32_t size);
    std::string GetCommand() const;
    bool IsValid(const unsigned char* expectedMagic) const;

    MessageStartChars magic;
    std::array<char, COMMAND_SIZE> command;
    uint32_t nMessageSize = 0;
    std::array<unsigned char, CHECKSUM_SIZE> checksum;

    template <typename S> void Serialize(S& s) const {
        s.write((const char*)magic.data(), 4);
        s.write(command.data(), COMMAND_SIZE);
        ::bcp::Serialize(s, nMessageSize);
        s.write((const char*)checksum.data(), 4);
    }
    template <typename S> void Unserialize(S& s) {
        s.read((char*)magic.data(), 4);
        s.read(command.data(), COMMAND_SIZE);
        ::bcp::Unserialize(s, nMessageSize);
        s.read((char*)checksum.data(), 4);
    }
};

enum GetDataMsg {
    UNDEFINED = 0,
    MSG_TX = 1,
    MSG_BLOCK = 2,
    MSG_FILTERED_BLOCK = 3, // getdata only: merkleblock + matched txs
    MSG_CMPCT_BLOCK = 4,    // getdata only: cmpctblock
};

class CInv {
public:
    CInv() {}
    CInv(int t, const uint256& h) : type(t), hash(h) {}
    int type = 0;
    uint256 hash;
    bool IsKnownType() const { return type >= 1 && type <= 4; }
    std::string GetCommand() const;
    std::string ToString() const { return GetCommand() + " " + hash.GetHex(); }
    friend bool operator<(const CInv& a, const CInv& b) { return a.type < b.type || (a.type == b.type && a.hash < b.hash); }
    friend bool operator==(const CInv& a, const CInv& b) { return a.type == b.type && a.hash == b.hash; }
    template <typename S> void Serialize(S& s) const {
        ::bcp::Serialize(s, type);
        ::bcp::Serialize(s, hash);
    }
    template <typename S> void Unserialize(S& s) {
        ::bcp::Unserialize(s, type);
        ::bcp::Unserialize(s, hash);
    }
};

// Checksum of a message payload: first 4 bytes of SHA256d.
void MessageChecksum(const unsigned char* p, size_t n, unsigned char out[4]);

// User agent with the excessive-block comment, e.g. "/Bitcoin Cash Plus:0.17.0(EB8.0)/"
// (reference src/net.cpp:3006-3030 getSubVersionEB/userAgent).
std::string UserAgent(uint64_t maxBlockSize);

} // namespace bcp
