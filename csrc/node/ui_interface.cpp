#include "node/ui_interface.h"
#include "util/util.h"

#include <cstdio>

namespace bcp {

CClientUIInterface uiInterface;

static int g_msgbox = 0, g_question = 0, g_init = 0;

static bool NoUIMessageBox(const std::string& message, const std::string& caption, unsigned style) {
    const bool fSecure = style & CClientUIInterface::SECURE;
    style &= ~CClientUIInterface::SECURE;
    std::string strCaption;
    switch (style) {
    case CClientUIInterface::MSG_ERROR: strCaption = "Error: "; break;
    case CClientUIInterface::MSG_WARNING: strCaption = "Warning: "; break;
    case CClientUIInterface::MSG_INFORMATION: strCaption = "Information: "; break;
    default: strCaption = caption + ": ";
    }
    if (!fSecure) LogPrintf("%s%s\n", strCaption.c_str(), message.c_str());
    fprintf(stderr, "%s%s\n", strCaption.c_str(), message.c_str());
    return false;
}

static bool NoUIQuestion(const std::string&, const std::string& noninteractive, const std::string& caption,
                         unsigned style) {
    return NoUIMessageBox(noninteractive, caption, style);
}

static void NoUIInitMessage(const std::string& message) { LogPrintf("init message: %s\n", message.c_str()); }

bool noui_connect() {
    if (g_msgbox) return false;
    g_msgbox = uiInterface.ThreadSafeMessageBox.connect(NoUIMessageBox);
    g_question = uiInterface.ThreadSafeQuestion.connect(NoUIQuestion);
    g_init = uiInterface.InitMessage.connect(NoUIInitMessage);
    return true;
}

void noui_disconnect() {
    if (!g_msgbox) return;
    uiInterface.ThreadSafeMessageBox.disconnect(g_msgbox);
    uiInterface.ThreadSafeQuestion.disconnect(g_question);
    uiInterface.InitMessage.disconnect(g_init);
    g_msgbox = g_question = g_init = 0;
}

bool InitError(const std::string& str) {
    uiInterface.ThreadSafeMessageBox(str, "", CClientUIInterface::MSG_ERROR);
    return false;
}

void InitWarning(const std::string& str) { uiInterface.ThreadSafeMessageBox(str, "", CClientUIInterface::MSG_WARNING); }

} // namespace bcp
