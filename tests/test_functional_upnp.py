"""UPnP port mapping (reference net.cpp ThreadMapPort over miniupnpc): against a fake
Internet Gateway Device (SSDP responder + description XML + SOAP control endpoint), a node
started with -upnp discovers the gateway, learns the external address (advertised in
getnetworkinfo localaddresses), maps its P2P port with AddPortMapping, and removes the
mapping with DeletePortMapping on shutdown."""
import http.server
import socket
import threading
import time

import pytest

from bitcoincashplus_amd.node.process import BcpdProcess

pytestmark = pytest.mark.functional

SERVICE = "urn:schemas-upnp-org:service:WANIPConnection:1"


class FakeIGD:
    def __init__(self, external_ip="93.184.216.34"):
        self.calls = []
        self.external_ip = external_ip
        igd = self

        class Handler(http.server.BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                body = (f"<?xml version=\"1.0\"?><root><device><deviceType>urn:schemas-upnp-org:device:"
                        f"InternetGatewayDevice:1</deviceType><deviceList><device><serviceList><service>"
                        f"<serviceType>{SERVICE}</serviceType><controlURL>/ctl/IPConn</controlURL>"
                        f"</service></serviceList></device></deviceList></device></root>").encode()
                self.send_response(200)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_POST(self):
                data = self.rfile.read(int(self.headers["Content-Length"])).decode()
                action = self.headers["SOAPAction"].strip('"').split("#")[1]
                igd.calls.append((action, data))
                out = ""
                if action == "GetExternalIPAddress":
                    out = f"<NewExternalIPAddress>{igd.external_ip}</NewExternalIPAddress>"
                body = (f"<?xml version=\"1.0\"?><s:Envelope xmlns:s=\"http://schemas.xmlsoap.org/soap/envelope/\">"
                        f"<s:Body><u:{action}Response xmlns:u=\"{SERVICE}\">{out}</u:{action}Response>"
                        f"</s:Body></s:Envelope>").encode()
                self.send_response(200)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.http = http.server.ThreadingHTTPServer(("127.0.0.1", 0), Handler)
        threading.Thread(target=self.http.serve_forever, daemon=True).start()
        self.udp = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.udp.bind(("127.0.0.1", 0))
        self.ssdp_port = self.udp.getsockname()[1]
        self.searches = []
        threading.Thread(target=self._ssdp, daemon=True).start()

    def _ssdp(self):
        while True:
            try:
                data, src = self.udp.recvfrom(2048)
            except OSError:
                return
            self.searches.append(data)
            if b"M-SEARCH" in data and b"InternetGatewayDevice" in data:
                loc = f"http://127.0.0.1:{self.http.server_address[1]}/rootDesc.xml"
                self.udp.sendto(f"HTTP/1.1 200 OK\r\nST: urn:schemas-upnp-org:device:InternetGatewayDevice:1\r\n"
                                f"LOCATION: {loc}\r\n\r\n".encode(), src)

    def close(self):
        self.http.shutdown()
        self.udp.close()


def test_upnp_maps_and_unmaps_port(tmp_path):
    igd = FakeIGD()
    n = BcpdProcess(str(tmp_path / "u"), extra_args=["-gpu=0", "-upnp", "-discover=1",
                                                       f"-upnpdiscover=127.0.0.1:{igd.ssdp_port}"])
    n.start()
    try:
        end = time.time() + 30
        while time.time() < end and not any(c[0] == "AddPortMapping" for c in igd.calls):
            time.sleep(0.2)
        actions = [c[0] for c in igd.calls]
        assert "GetExternalIPAddress" in actions and "AddPortMapping" in actions
        add = next(c[1] for c in igd.calls if c[0] == "AddPortMapping")
        assert f"<NewExternalPort>{n.p2p_port}</NewExternalPort>" in add
        assert "<NewProtocol>TCP</NewProtocol>" in add and "<NewInternalClient>127.0.0.1</NewInternalClient>" in add
        locals_ = n.rpc.getnetworkinfo()["localaddresses"]
        assert any(a["address"] == "93.184.216.34" for a in locals_)
    finally:
        n.stop()
        igd.close()
    assert igd.calls[-1][0] == "DeletePortMapping"
