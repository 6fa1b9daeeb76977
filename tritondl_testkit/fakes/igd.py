"""Fake UPnP Internet Gateway Device for tests: an SSDP responder (unicast,
on loopback) plus the HTTP device description and a WANIPConnection:1 SOAP
control endpoint that keeps a port-mapping table."""

from __future__ import annotations

import asyncio
import xml.etree.ElementTree as ET

from aiohttp import web

ST = "urn:schemas-upnp-org:device:InternetGatewayDevice:1"
SVC = "urn:schemas-upnp-org:service:WANIPConnection:1"

_DESC = """<?xml version="1.0"?>
<root xmlns="urn:schemas-upnp-org:device-1-0">
 <specVersion><major>1</major><minor>0</minor></specVersion>
 <device>
  <deviceType>urn:schemas-upnp-org:device:InternetGatewayDevice:1</deviceType>
  <friendlyName>fake gateway</friendlyName>
  <serviceList><service>
   <serviceType>urn:schemas-upnp-org:service:Layer3Forwarding:1</serviceType>
   <controlURL>/l3f</controlURL></service></serviceList>
  <deviceList><device>
   <deviceType>urn:schemas-upnp-org:device:WANDevice:1</deviceType>
   <deviceList><device>
    <deviceType>urn:schemas-upnp-org:device:WANConnectionDevice:1</deviceType>
    <serviceList><service>
     <serviceType>urn:schemas-upnp-org:service:WANIPConnection:1</serviceType>
     <serviceId>urn:upnp-org:serviceId:WANIPConn1</serviceId>
     <controlURL>/ctl/IPConn</controlURL>
     <SCPDURL>/WANIPCn.xml</SCPDURL>
    </service></serviceList>
   </device></deviceList>
  </device></deviceList>
 </device>
</root>"""


def _fault(code: int, desc: str) -> web.Response:
    body = ('<?xml version="1.0"?><s:Envelope xmlns:s="http://schemas.xmlsoap.org/soap/envelope/"><s:Body>'
            '<s:Fault><faultcode>s:Client</faultcode><faultstring>UPnPError</faultstring><detail>'
            '<UPnPError xmlns="urn:schemas-upnp-org:control-1-0">'
            f'<errorCode>{code}</errorCode><errorDescription>{desc}</errorDescription>'
            '</UPnPError></detail></s:Fault></s:Body></s:Envelope>')
    return web.Response(status=500, body=body.encode(), content_type="text/xml")


class FakeIGD:
    def __init__(self, external_ip: str = "203.0.113.7") -> None:
        self.external_ip = external_ip
        self.mappings: dict[tuple[int, str], dict] = {}
        self.actions: list[str] = []
        self.searches = 0
        self._runner: web.AppRunner | None = None
        self._udp: asyncio.DatagramTransport | None = None
        self.http_port = 0
        self.ssdp_port = 0

    @property
    def ssdp_addr(self) -> tuple[str, int]:
        return ("127.0.0.1", self.ssdp_port)

    async def start(self) -> "FakeIGD":
        app = web.Application()
        app.router.add_get("/rootDesc.xml", self._desc)
        app.router.add_post("/ctl/IPConn", self._control)
        self._runner = web.AppRunner(app)
        await self._runner.setup()
        site = web.TCPSite(self._runner, "127.0.0.1", 0)
        await site.start()
        self.http_port = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
        igd = self

        class P(asyncio.DatagramProtocol):
            def connection_made(self, tr):
                self.tr = tr

            def datagram_received(self, data, addr):
                if not data.startswith(b"M-SEARCH") or ST.encode() not in data:
                    return
                igd.searches += 1
                self.tr.sendto(("HTTP/1.1 200 OK\r\nCACHE-CONTROL: max-age=120\r\n"
                                f"LOCATION: http://127.0.0.1:{igd.http_port}/rootDesc.xml\r\n"
                                f"ST: {ST}\r\nUSN: uuid:fake::{ST}\r\n\r\n").encode(), addr)

        loop = asyncio.get_running_loop()
        self._udp, _ = await loop.create_datagram_endpoint(P, local_addr=("127.0.0.1", 0))
        self.ssdp_port = self._udp.get_extra_info("sockname")[1]
        return self

    async def stop(self) -> None:
        if self._udp is not None:
            self._udp.close()
        if self._runner is not None:
            await self._runner.cleanup()

    async def _desc(self, request: web.Request) -> web.Response:
        return web.Response(body=_DESC.encode(), content_type="text/xml")

    async def _control(self, request: web.Request) -> web.Response:
        action = request.headers.get("SOAPAction", "").strip('"').rpartition("#")[2]
        self.actions.append(action)
        root = ET.fromstring(await request.read())
        args: dict[str, str] = {}
        for el in root.iter():
            if el.tag.endswith(action):
                args = {c.tag.rsplit("}", 1)[-1]: (c.text or "") for c in el}
        if action == "GetExternalIPAddress":
            return self._ok(action, {"NewExternalIPAddress": self.external_ip})
        if action == "AddPortMapping":
            key = (int(args["NewExternalPort"]), args["NewProtocol"])
            cur = self.mappings.get(key)
            if cur is not None and cur["client"] != args["NewInternalClient"]:
                return _fault(718, "ConflictInMappingEntry")
            self.mappings[key] = {"client": args["NewInternalClient"], "internal_port": int(args["NewInternalPort"]),
                                  "desc": args.get("NewPortMappingDescription", ""),
                                  "lease": int(args.get("NewLeaseDuration", "0") or 0)}
            return self._ok(action, {})
        if action == "DeletePortMapping":
            key = (int(args["NewExternalPort"]), args["NewProtocol"])
            if key not in self.mappings:
                return _fault(714, "NoSuchEntryInArray")
            del self.mappings[key]
            return self._ok(action, {})
        return _fault(401, "Invalid Action")

    def _ok(self, action: str, out: dict[str, str]) -> web.Response:
        inner = "".join(f"<{k}>{v}</{k}>" for k, v in out.items())
        body = ('<?xml version="1.0"?><s:Envelope xmlns:s="http://schemas.xmlsoap.org/soap/envelope/"><s:Body>'
                f'<u:{action}Response xmlns:u="{SVC}">{inner}</u:{action}Response></s:Body></s:Envelope>')
        return web.Response(body=body.encode(), content_type="text/xml")
