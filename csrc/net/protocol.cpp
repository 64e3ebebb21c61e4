#include "net/protocol.h"
#include "crypto/hashes.h"
#include "util/strencodings.h"
#include "util/util.h"
#include "node/miner.h"

#include <algorithm>

namespace bcp {

namespace NetMsgType {
const char* VERSION = "version";
const char* VERACK = "verack";
const char* ADDR = "addr";
const char* INV = "inv";
const char* GETDATA = "getdata";
const char* MERKLEBLOCK = "merkleblock";
const char* GETBLOCKS = "getblocks";
const char* GETHEADERS = "getheaders";
const char* TX = "tx";
const char* HEADERS = "headers";
const char* BLOCK = "block";
const char* GETADDR = "getaddr";
const char* MEMPOOL = "mempool";
const char* PING = "ping";
const char* PONG = "pong";
const char* NOTFOUND = "notfound";
const char* FILTERLOAD = "filterload";
const char* FILTERADD = "filteradd";
const char* FILTERCLEAR = "filterclear";
const char* REJECT = "reject";
const char* SENDHEADERS = "sendheaders";
const char* FEEFILTER = "feefilter";
const char* SENDCMPCT = "sendcmpct";
const char* CMPCTBLOCK = "cmpctblock";
const char* GETBLOCKTXN = "getblocktxn";
const char* BLOCKTXN = "blocktxn";
} // namespace NetMsgType

const std::vector<std::string>& GetAllNetMessageTypes() {
    using namespace NetMsgType;
    static const std::vector<std::string> all = {
        VERSION, VERACK,     ADDR,        INV,         GETDATA,  MERKLEBLOCK, GETBLOCKS,  GETHEADERS, TX,
        HEADERS, BLOCK,      GETADDR,     MEMPOOL,     PING,     PONG,        NOTFOUND,   FILTERLOAD, FILTERADD,
        FILTERCLEAR, REJECT, SENDHEADERS, FEEFILTER,   SENDCMPCT, CMPCTBLOCK, GETBLOCKTXN, BLOCKTXN};
    return all;
}

CMessageHeader::CMessageHeader(const unsigned char* start, const char* cmd, uint32_t size) : nMessageSize(size) {
    memcpy(magic.data(), start, 4);
    command.fill(0);
    memcpy(command.data(), cmd, std::min(strlen(cmd), COMMAND_SIZE));
    checksum.fill(0);
}

std::string CMessageHeader::GetCommand() const {
    return std::string(command.data(), strnlen(command.data(), COMMAND_SIZE));
}

bool CMessageHeader::IsValid(const unsigned char* expectedMagic) const {
    if (memcmp(magic.data(), expectedMagic, 4) != 0) return false;
    // command: printable chars, then only NULs
    bool end = false;
    for (char c : command) {
        if (end) {
            if (c != 0) return false;
        } else if (c == 0) {
            end = true;
        } else if (c < ' ' || c > 0x7E) {
            return false;
        }
    }
    return nMessageSize <= MAX_PROTOCOL_MESSAGE_LENGTH;
}

std::string CInv::GetCommand() const {
    switch (type) {
    case MSG_TX: return NetMsgType::TX;
    case MSG_BLOCK: return NetMsgType::BLOCK;
    case MSG_FILTERED_BLOCK: return NetMsgType::MERKLEBLOCK;
    case MSG_CMPCT_BLOCK: return NetMsgType::CMPCTBLOCK;
    default: return strprintf("unknown(%d)", type);
    }
}

void MessageChecksum(const unsigned char* p, size_t n, unsigned char out[4]) {
    unsigned char h[32];
    Sha256d(p, n, h);
    memcpy(out, h, 4);
}

std::string UserAgent(uint64_t maxBlockSize) {
    std::vector<std::string> comments{"EB" + GetSubVersionEB(maxBlockSize)};
    for (const std::string& c : gArgs.GetArgs("-uacomment")) comments.push_back(SanitizeString(c));
    std::string ua = FormatSubVersion(CLIENT_NAME, CLIENT_VERSION, comments);
    if (ua.size() > MAX_SUBVERSION_LENGTH) {
        // cut to the limit, still closed like a version string (reference net.cpp:3041-3049)
        LogPrintf("Total length of network version string (%i) exceeds maximum length (%i). Reduce the number or "
                  "size of uacomments. String has been resized to the max length allowed.\n",
                  (int)ua.size(), (int)MAX_SUBVERSION_LENGTH);
        ua.resize(MAX_SUBVERSION_LENGTH - 2);
        ua += ")/";
    }
    return ua;
}

} // namespace bcp
