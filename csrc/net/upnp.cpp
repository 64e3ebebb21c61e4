// UPnP port mapping (reference src/net.cpp ThreadMapPort / MapPort, built on miniupnpc:
// upnpDiscover, UPNP_GetValidIGD, UPNP_GetExternalIPAddress, UPNP_AddPortMapping every 20
// minutes, UPNP_DeletePortMapping at shutdown). Self-contained here: SSDP M-SEARCH for an
// InternetGatewayDevice, HTTP GET of its description, SOAP calls to the WANIPConnection (or
// WANPPPConnection) control URL. -upnp turns it on; the external address the gateway reports is
// advertised like an address learned by UPnP (LOCAL_UPNP). -upnpdiscover=<ip:port> sends the
// M-SEARCH to a unicast address instead of 239.255.255.250:1900 (tests, routed setups).
#include "net/net.h"
#include "net/netaddress.h"
#include "util/strencodings.h"
#include "util/util.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>

namespace bcp {

namespace {

std::thread g_upnpThread;
std::mutex g_upnpMu;
std::condition_variable g_upnpCv;
std::atomic<bool> g_upnpStop{false};

std::string Lower(std::string s) {
    for (char& c : s) c = (char)tolower((unsigned char)c);
    return s;
}

// Text between <tag> and </tag> (first occurrence at or after `from`), namespace prefixes ignored.
std::string XmlValue(const std::string& xml, const std::string& tag, size_t from = 0, size_t* endOut = nullptr) {
    size_t p = from;
    while (true) {
        p = xml.find(tag, p);
        if (p == std::string::npos) return "";
        const size_t lt = xml.rfind('<', p);
        const size_t gt = xml.find('>', p);
        if (lt != std::string::npos && gt != std::string::npos && xml[lt + 1] != '/' &&
            (p == lt + 1 || xml[p - 1] == ':') && (xml[p + tag.size()] == '>' || xml[p + tag.size()] == ' ')) {
            const size_t close = xml.find("</", gt);
            if (close == std::string::npos) return "";
            if (endOut) *endOut = close;
            return xml.substr(gt + 1, close - gt - 1);
        }
        p += tag.size();
    }
}

struct Url {
    std::string host, path;
    uint16_t port = 80;
};
bool ParseUrl(const std::string& u, Url& out) {
    if (u.compare(0, 7, "http://") != 0) return false;
    const size_t slash = u.find('/', 7);
    const std::string hostport = u.substr(7, slash == std::string::npos ? std::string::npos : slash - 7);
    out.path = slash == std::string::npos ? "/" : u.substr(slash);
    int port = 80;
    SplitHostPort(hostport, port, out.host);
    out.port = (uint16_t)port;
    return !out.host.empty();
}

// One blocking HTTP/1.1 request; returns the body (empty on failure). localAddr gets the
// source address of the connection (our LAN address as the gateway sees it).
std::string HttpRequest(const Url& url, const std::string& method, const std::string& extraHeaders,
                        const std::string& body, std::string* localAddr = nullptr) {
    CService svc = LookupNumeric(url.host, url.port);
    struct sockaddr_storage ss;
    socklen_t len = sizeof(ss);
    if (!svc.GetSockAddr((struct sockaddr*)&ss, &len)) return "";
    const int fd = socket(((struct sockaddr*)&ss)->sa_family, SOCK_STREAM, IPPROTO_TCP);
    if (fd < 0) return "";
    struct timeval tv = {5, 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    if (connect(fd, (struct sockaddr*)&ss, len) != 0) {
        close(fd);
        return "";
    }
    if (localAddr) {
        struct sockaddr_storage me;
        socklen_t ml = sizeof(me);
        char buf[INET6_ADDRSTRLEN] = {};
        if (getsockname(fd, (struct sockaddr*)&me, &ml) == 0 && me.ss_family == AF_INET)
            inet_ntop(AF_INET, &((struct sockaddr_in*)&me)->sin_addr, buf, sizeof(buf));
        *localAddr = buf;
    }
    const std::string req = method + " " + url.path + " HTTP/1.1\r\nHost: " + url.host + ":" +
                            std::to_string(url.port) + "\r\nConnection: close\r\n" + extraHeaders +
                            "Content-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
    if (send(fd, req.data(), req.size(), MSG_NOSIGNAL) != (ssize_t)req.size()) {
        close(fd);
        return "";
    }
    std::string resp;
    char buf[4096];
    ssize_t n;
    while ((n = recv(fd, buf, sizeof(buf), 0)) > 0 && resp.size() < (1 << 20)) resp.append(buf, (size_t)n);
    close(fd);
    const size_t hdrEnd = resp.find("\r\n\r\n");
    if (hdrEnd == std::string::npos || resp.compare(0, 7, "HTTP/1.") != 0 || resp.compare(8, 4, " 200") != 0)
        return "";
    return resp.substr(hdrEnd + 4);
}

// SSDP search; returns the LOCATION of the first InternetGatewayDevice that answers.
std::string Discover(int timeoutMs) {
    const std::string target = gArgs.GetArg("-upnpdiscover", "239.255.255.250:1900");
    CService dst = LookupNumeric(target, 1900);
    struct sockaddr_storage ss;
    socklen_t len = sizeof(ss);
    if (!dst.GetSockAddr((struct sockaddr*)&ss, &len)) return "";
    const int fd = socket(AF_INET, SOCK_DGRAM, IPPROTO_UDP);
    if (fd < 0) return "";
    const std::string msg =
        "M-SEARCH * HTTP/1.1\r\nHOST: 239.255.255.250:1900\r\nMAN: \"ssdp:discover\"\r\nMX: 2\r\n"
        "ST: urn:schemas-upnp-org:device:InternetGatewayDevice:1\r\n\r\n";
    sendto(fd, msg.data(), msg.size(), 0, (struct sockaddr*)&ss, len);
    std::string location;
    const int64_t deadline = GetTimeMillis() + timeoutMs;
    while (location.empty() && GetTimeMillis() < deadline && !g_upnpStop) {
        struct pollfd p = {fd, POLLIN, 0};
        if (poll(&p, 1, 200) <= 0) continue;
        char buf[2048];
        const ssize_t n = recv(fd, buf, sizeof(buf) - 1, 0);
        if (n <= 0) continue;
        const std::string reply(buf, (size_t)n);
        for (size_t pos = 0; pos < reply.size();) {
            const size_t eol = reply.find("\r\n", pos);
            const std::string line = reply.substr(pos, eol == std::string::npos ? std::string::npos : eol - pos);
            if (Lower(line).compare(0, 9, "location:") == 0) {
                location = line.substr(9);
                while (!location.empty() && location[0] == ' ') location.erase(0, 1);
                break;
            }
            if (eol == std::string::npos) break;
            pos = eol + 2;
        }
    }
    close(fd);
    return location;
}

struct Igd {
    Url control;
    std::string serviceType;
    std::string lanAddr;
};

bool FindIgd(const std::string& location, Igd& igd) {
    Url desc;
    if (!ParseUrl(location, desc)) return false;
    const std::string xml = HttpRequest(desc, "GET", "", "", &igd.lanAddr);
    if (xml.empty()) return false;
    // first WAN connection service (IP preferred over PPP)
    for (const char* want : {"urn:schemas-upnp-org:service:WANIPConnection:1",
                             "urn:schemas-upnp-org:service:WANPPPConnection:1"}) {
        const size_t at = xml.find(want);
        if (at == std::string::npos) continue;
        std::string ctrl = XmlValue(xml, "controlURL", at);
        if (ctrl.empty()) continue;
        if (ctrl.compare(0, 7, "http://") != 0) {
            std::string base = XmlValue(xml, "URLBase");
            if (base.empty()) base = "http://" + desc.host + ":" + std::to_string(desc.port);
            while (!base.empty() && base.back() == '/') base.pop_back();
            ctrl = base + (ctrl[0] == '/' ? "" : "/") + ctrl;
        }
        if (!ParseUrl(ctrl, igd.control)) continue;
        igd.serviceType = want;
        return true;
    }
    return false;
}

std::string Soap(const Igd& igd, const std::string& action, const std::string& args) {
    const std::string body = "<?xml version=\"1.0\"?>\r\n<s:Envelope xmlns:s=\"http://schemas.xmlsoap.org/soap/"
                             "envelope/\" s:encodingStyle=\"http://schemas.xmlsoap.org/soap/encoding/\"><s:Body>"
                             "<u:" + action + " xmlns:u=\"" + igd.serviceType + "\">" + args + "</u:" + action +
                             "></s:Body></s:Envelope>\r\n";
    return HttpRequest(igd.control, "POST",
                       "Content-Type: text/xml; charset=\"utf-8\"\r\nSOAPAction: \"" + igd.serviceType + "#" +
                           action + "\"\r\n",
                       body);
}

void ThreadMapPort(int port) {
    RenameThread("bcp-upnp");
    const std::string location = Discover(2000);
    Igd igd;
    if (location.empty() || !FindIgd(location, igd)) {
        LogPrintf("No valid UPnP IGDs found\n");
        return;
    }
    const std::string ext = XmlValue(Soap(igd, "GetExternalIPAddress", ""), "NewExternalIPAddress");
    if (!ext.empty()) {
        LogPrintf("UPnP: ExternalIPAddress = %s\n", ext.c_str());
        CService extAddr = LookupNumeric(ext, port);
        if (extAddr.IsValid()) AddLocal(extAddr, LOCAL_UPNP);
    } else {
        LogPrintf("UPnP: GetExternalIPAddress failed.\n");
    }
    const std::string sport = std::to_string(port);
    const std::string mapArgs = "<NewRemoteHost></NewRemoteHost><NewExternalPort>" + sport +
                                "</NewExternalPort><NewProtocol>TCP</NewProtocol><NewInternalPort>" + sport +
                                "</NewInternalPort><NewInternalClient>" + igd.lanAddr +
                                "</NewInternalClient><NewEnabled>1</NewEnabled><NewPortMappingDescription>"
                                "Bitcoin Cash Plus " + FormatFullVersion() +
                                "</NewPortMappingDescription><NewLeaseDuration>0</NewLeaseDuration>";
    std::unique_lock<std::mutex> lk(g_upnpMu);
    while (!g_upnpStop) {
        lk.unlock();
        // the reference answers "AddPortMapping" errors with a log line and retries next round
        if (Soap(igd, "AddPortMapping", mapArgs).empty())
            LogPrintf("AddPortMapping(%s, %s, %s) failed\n", sport.c_str(), sport.c_str(), igd.lanAddr.c_str());
        else
            LogPrintf("UPnP Port Mapping successful.\n");
        lk.lock();
        g_upnpCv.wait_for(lk, std::chrono::minutes(20), [] { return g_upnpStop.load(); });
    }
    lk.unlock();
    Soap(igd, "DeletePortMapping",
         "<NewRemoteHost></NewRemoteHost><NewExternalPort>" + sport + "</NewExternalPort><NewProtocol>TCP</NewProtocol>");
    LogPrintf("UPNP_DeletePortMapping() done\n");
}

} // namespace

void StopMapPort();
void StartMapPort(int port) {
    StopMapPort();
    g_upnpStop = false;
    g_upnpThread = std::thread(ThreadMapPort, port);
}

void StopMapPort() {
    if (!g_upnpThread.joinable()) return;
    {
        std::lock_guard<std::mutex> l(g_upnpMu);
        g_upnpStop = true;
    }
    g_upnpCv.notify_all();
    g_upnpThread.join();
}

} // namespace bcp
