"""UPnP IGD port forwarding (anacrolix default-config behaviour behind the
reference's ``torrent.NewDefaultClientConfig()``, torrent.go:40): SSDP
discovery, device description walk, SOAP AddPortMapping /
GetExternalIPAddress / DeletePortMapping against a fake gateway, caching,
and the Torrent's listen-port lifecycle."""

import asyncio
import socket

from tritondl_testkit.fakes.igd import FakeIGD
from tritondl.fetch.bt import portfwd
from tritondl.fetch.bt.torrent import Torrent, TorrentConfig


def run(coro, timeout=30):
    return asyncio.run(asyncio.wait_for(coro, timeout))


def test_forward_and_unmap_tcp_udp():
    async def main():
        igd = await FakeIGD().start()
        pf = portfwd.PortForwarder(51413, ssdp_addr=igd.ssdp_addr, timeout=1.0)
        assert await pf.start()
        assert set(igd.mappings) == {(51413, "TCP"), (51413, "UDP")}
        m = igd.mappings[(51413, "TCP")]
        assert m["client"] == "127.0.0.1" and m["internal_port"] == 51413 and "tritondl" in m["desc"]
        assert pf.external_ip == "203.0.113.7"
        assert pf.gateway.control_url.endswith("/ctl/IPConn")
        await pf.close()
        assert igd.mappings == {}
        # discovery is cached per process: a second forwarder does not search again
        pf2 = portfwd.PortForwarder(6881, ssdp_addr=igd.ssdp_addr, timeout=1.0)
        assert await pf2.start() and igd.searches == 1
        await pf2.close()
        await igd.stop()
    run(main())


def test_mapping_conflict_is_reported_not_fatal():
    async def main():
        igd = await FakeIGD().start()
        igd.mappings[(7000, "TCP")] = {"client": "10.9.9.9", "internal_port": 7000, "desc": "other", "lease": 0}
        pf = portfwd.PortForwarder(7000, ssdp_addr=igd.ssdp_addr, timeout=1.0)
        assert await pf.start()                    # UDP mapped, TCP refused (718 ConflictInMappingEntry)
        assert pf.mapped == ["UDP"] and igd.mappings[(7000, "TCP")]["client"] == "10.9.9.9"
        await pf.close()
        assert (7000, "UDP") not in igd.mappings and (7000, "TCP") in igd.mappings
        await igd.stop()
    run(main())


def test_no_gateway_times_out_quietly_and_is_cached():
    async def main():
        silent = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        silent.bind(("127.0.0.1", 0))
        addr = silent.getsockname()
        t0 = asyncio.get_running_loop().time()
        assert await portfwd.discover(addr, timeout=0.3) is None
        assert await portfwd.discover(addr, timeout=0.3) is None        # cached: no second wait
        assert asyncio.get_running_loop().time() - t0 < 0.55
        pf = portfwd.PortForwarder(1234, ssdp_addr=addr, timeout=0.3)
        assert not await pf.start()
        await pf.close()
        silent.close()
    run(main())


def test_torrent_forwards_its_listen_port_for_its_lifetime(tmp_path):
    async def main():
        igd = await FakeIGD().start()
        t = Torrent(b"\x11" * 20, str(tmp_path), TorrentConfig(listen_host="127.0.0.1", upnp=True,
                                                               upnp_ssdp=igd.ssdp_addr))
        await t.start()
        for _ in range(500):                 # SSDP + SOAP round trips: slow under a loaded CI box
            if len(igd.mappings) == 2:
                break
            await asyncio.sleep(0.02)
        assert set(igd.mappings) == {(t.port, "TCP"), (t.port, "UDP")}
        await t.close()
        assert igd.mappings == {}
        await igd.stop()
    run(main())
