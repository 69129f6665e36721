"""Interface and broadcast-socket plumbing of a Kaboodle instance (src/networking.rs:12-130), for the bridge
between a simulated mesh and real instances (kaboodle_amd.bridge).

    best_available_interface()                 -> Interface   (networking.rs:12-27; IPv6 preferred)
    non_loopback_interfaces()                  -> [Interface] (networking.rs:123-130)
    create_broadcast_sockets(interface, port)  -> (in_sock, out_sock, broadcast_addr)   (networking.rs:29-121)

IPv4: one SO_BROADCAST socket bound to 0.0.0.0:<port> serves both directions and sends to
255.255.255.255:<port>.  IPv6: the inbound socket joins the link-local multicast group ff02::1213:1989
on the interface and binds [::]:<port>; the outbound one names the interface as its multicast interface
and binds [::]:0.  Sockets are non-blocking with SO_REUSEADDR and SO_REUSEPORT, as the reference sets them.
"""
from __future__ import annotations

import ipaddress
import socket
import struct
from dataclasses import dataclass

MULTICAST_V6 = "ff02::1213:1989"          # networking.rs:80: link-local scope, Kaboodle's group id


class NoAvailableInterfaces(OSError):
    """KaboodleError::NoAvailableInterfaces (src/errors.rs)."""


class UnableToFindInterfaceNumber(OSError):
    """KaboodleError::UnableToFindInterfaceNumber (src/errors.rs)."""


@dataclass(frozen=True)
class Interface:
    """if_addrs::Interface: name, address, and the OS interface index (needed for IPv6 multicast)."""
    name: str
    ip: str
    index: int | None = None

    @property
    def is_ipv6(self) -> bool:
        return ipaddress.ip_address(self.ip.split("%")[0]).version == 6

    def is_loopback(self) -> bool:
        return ipaddress.ip_address(self.ip.split("%")[0]).is_loopback


def _all_interfaces() -> list[Interface]:
    import psutil
    index = {name: idx for idx, name in socket.if_nameindex()}
    out = []
    for name, addrs in psutil.net_if_addrs().items():
        for a in addrs:
            if a.family in (socket.AF_INET, socket.AF_INET6):
                out.append(Interface(name, a.address.split("%")[0], index.get(name)))
    return out


def non_loopback_interfaces() -> list[Interface]:
    return [i for i in _all_interfaces() if not i.is_loopback()]


def best_available_interface() -> Interface:
    """The first IPv6 non-loopback interface, else the first IPv4 one (networking.rs:12-27)."""
    nl = non_loopback_interfaces()
    v6 = [i for i in nl if i.is_ipv6]
    if v6:
        return v6[0]
    if nl:
        return nl[0]
    raise NoAvailableInterfaces("no non-loopback network interface")


def _reuse(sock: socket.socket) -> None:
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    if hasattr(socket, "SO_REUSEPORT"):
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)


def create_broadcast_sockets(interface: Interface, port: int):
    """(broadcast_in_sock, broadcast_out_sock, broadcast_addr) as networking.rs:29-121 builds them."""
    if not interface.is_ipv6:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM, socket.IPPROTO_UDP)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_BROADCAST, 1)
        s.setblocking(False)
        _reuse(s)
        s.bind(("0.0.0.0", port))
        # one socket both ways; two handles for the callers' symmetry (networking.rs:56-61)
        return s, s.dup(), ("255.255.255.255", port)
    if interface.index is None:
        raise UnableToFindInterfaceNumber(interface.name)
    group = socket.inet_pton(socket.AF_INET6, MULTICAST_V6)
    sin = socket.socket(socket.AF_INET6, socket.SOCK_DGRAM, socket.IPPROTO_UDP)
    sin.setsockopt(socket.IPPROTO_IPV6, socket.IPV6_JOIN_GROUP, group + struct.pack("@I", interface.index))
    sin.setblocking(False)
    sin.setsockopt(socket.IPPROTO_IPV6, socket.IPV6_V6ONLY, 1)
    _reuse(sin)
    sin.bind(("::", port))
    sout = socket.socket(socket.AF_INET6, socket.SOCK_DGRAM, socket.IPPROTO_UDP)
    sout.setsockopt(socket.IPPROTO_IPV6, socket.IPV6_MULTICAST_IF, interface.index)
    sout.setblocking(False)
    _reuse(sout)
    sout.bind(("::", 0))
    return sin, sout, (MULTICAST_V6, port)
