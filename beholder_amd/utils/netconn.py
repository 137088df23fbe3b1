"""Hand an established plain-TCP asyncio connection over to a native ``NetConn``.

(HTTP sink connections do not go through here: they are connected by the NetConn itself,
``ops.native.netconn_connect``; Postgres connections, authenticated on asyncio first, are.)

``ops/csrc/py_netconn.cpp`` drives a socket straight from the event loop's selector and does
the protocol work (HTTP/1.1 response parsing, Postgres reply matching) in C, so a reply costs
no Python-level transport / protocol frames. Connections are opened, TLS-wrapped and
authenticated with ordinary asyncio transports; a connection that ends up as plain TCP is then
adopted: its socket is duplicated, the asyncio transport is aborted (the duplicate keeps the TCP
connection open) and the duplicate goes to the ``NetConn``. TLS connections stay on asyncio.

``BEHOLDER_NATIVE_IO=0`` is the one switch for all native I/O (debugging, A/B runs): every
connection stays on an asyncio transport (TLS included), the H1 client and the Postgres pool take
their Python request paths, and replies complete plain ``asyncio.Future``s (read at import).
"""
from __future__ import annotations

import os
import socket
from typing import Optional

from ..ops import native

NetConn = native.NetConn


def enabled() -> bool:
    """Native I/O on (``BEHOLDER_NATIVE_IO`` is not ``0``)."""
    return os.environ.get("BEHOLDER_NATIVE_IO", "1") != "0"


def adopt(transport) -> Optional[int]:
    """A duplicate of ``transport``'s socket fd, with the transport aborted; None (transport
    untouched) when it is not a plain TCP socket transport with an empty write buffer."""
    if not enabled() or transport is None or transport.is_closing():
        return None
    if transport.get_extra_info("sslcontext") is not None or transport.get_extra_info("ssl_object") is not None:
        return None
    sock = transport.get_extra_info("socket")
    if sock is None or sock.family not in (socket.AF_INET, socket.AF_INET6) or sock.type != socket.SOCK_STREAM:
        return None
    if transport.get_write_buffer_size():
        return None
    fd = os.dup(sock.fileno())
    os.set_blocking(fd, False)
    transport.abort()  # the protocol's connection_lost for this transport must be ignored
    return fd
