"""Built-in host-local IPAM (the reference delegates to the `host-local` CNI plugin binary,
sriov.go ipam.ExecAdd; no CNI plugin binaries exist here, so the same allocation semantics are
implemented directly: one file per allocated IP under <dir>/<network>/, holding the owner)."""
from __future__ import annotations

import ipaddress
import os
import threading


class HostLocalIpam:
    def __init__(self, data_dir: str = "/var/lib/cni/networks"):
        self.dir = data_dir
        self._lock = threading.Lock()
        self.subnets: dict[str, str] = {}

    def configure(self, network: str, subnet: str) -> None:
        self.subnets[network] = subnet

    def _ndir(self, network: str) -> str:
        d = os.path.join(self.dir, network)
        os.makedirs(d, exist_ok=True)
        return d

    def allocate(self, network: str, container_id: str, ifname: str) -> dict:
        subnet = ipaddress.ip_network(self.subnets.get(network, "10.56.217.0/24"))
        owner = f"{container_id}\n{ifname}"
        with self._lock:
            d = self._ndir(network)
            for f in os.listdir(d):
                p = os.path.join(d, f)
                if os.path.isfile(p) and open(p).read() == owner:
                    return {"address": f"{f}/{subnet.prefixlen}", "gateway": str(next(subnet.hosts()))}
            hosts = list(subnet.hosts())
            for ip in hosts[1:]:  # first host = gateway
                p = os.path.join(d, str(ip))
                try:
                    fd = os.open(p, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644)
                except FileExistsError:
                    continue
                with os.fdopen(fd, "w") as fh:
                    fh.write(owner)
                return {"address": f"{ip}/{subnet.prefixlen}", "gateway": str(hosts[0])}
        raise RuntimeError(f"no IP addresses available in range set: {subnet}")

    def release(self, network: str, container_id: str, ifname: str) -> None:
        owner = f"{container_id}\n{ifname}"
        with self._lock:
            d = self._ndir(network)
            for f in os.listdir(d):
                p = os.path.join(d, f)
                if os.path.isfile(p) and open(p).read() == owner:
                    os.unlink(p)
