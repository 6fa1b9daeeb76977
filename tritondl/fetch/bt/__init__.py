"""BitTorrent stack (reference C7 + the anacrolix/torrent capabilities it
uses): bencode, metainfo/magnets, peer wire + ut_metadata, HTTP/UDP trackers,
mainline DHT, file storage + completion DB + batch resume verification,
swarm session, and the ``torrent`` downloader plug-in."""
