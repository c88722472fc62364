"""CNI request / pod-request / NetConf types (wire format of the dpu-cni HTTP protocol).

Reference: dpu-cni/pkgs/cnitypes/cnitypes.go:13-135.  ``Request`` is what the shim POSTs:
``{"env": {...CNI_* vars...}, "config": <base64 stdin bytes>, <DeviceInfo fields>}`` — Go's
encoding/json renders []byte as base64, so the same JSON is produced here.
"""
from __future__ import annotations

import base64
import json
import threading
import time
from dataclasses import dataclass, field

DAEMON_BASE_DIR = "/var/run/dpu-daemon/"
SERVER_SOCKET_PATH = DAEMON_BASE_DIR + "dpu-cni/dpu-cni-server.sock"

CNI_ADD, CNI_UPDATE, CNI_DEL, CNI_CHECK = "ADD", "UPDATE", "DEL", "CHECK"
PROTO_8021Q, PROTO_8021AD = "802.1q", "802.1ad"
VLAN_PROTO_INT = {PROTO_8021Q: 33024, PROTO_8021AD: 34984}
SUPPORTED_VERSIONS = ["0.3.0", "0.3.1", "0.4.0", "1.0.0"]


class CNIError(Exception):
    def __init__(self, msg: str, code: int = 999):
        super().__init__(msg)
        self.code = code

    def to_json(self, version: str = "1.0.0") -> dict:
        return {"cniVersion": version, "code": self.code, "msg": str(self)}


@dataclass
class Request:
    env: dict[str, str] = field(default_factory=dict)
    config: bytes = b""
    device_info: dict = field(default_factory=dict)

    def to_json(self) -> bytes:
        d = {"env": self.env, "config": base64.b64encode(self.config).decode()}
        d.update(self.device_info)
        return json.dumps(d).encode()

    @classmethod
    def from_json(cls, b: bytes) -> "Request":
        d = json.loads(b)
        cfg = d.pop("config", "") or ""
        env = d.pop("env", {}) or {}
        return cls(env=env, config=base64.b64decode(cfg) if cfg else b"", device_info=d)


@dataclass
class VfState:
    HostIFName: str = ""
    SpoofChk: bool = False
    Trust: bool = False
    AdminMAC: str = ""
    EffectiveMAC: str = ""
    Vlan: int = 0
    VlanQoS: int = 0
    VlanProto: int = 0
    MinTxRate: int = 0
    MaxTxRate: int = 0
    LinkState: int = 0


@dataclass
class NetConf:
    """CNI network config plus the SR-IOV fields (cnitypes.go NetConf)."""
    cniVersion: str = "0.4.0"
    name: str = ""
    type: str = ""
    ipam: dict = field(default_factory=dict)
    dns: dict = field(default_factory=dict)
    prevResult: dict | None = None
    OrigVfState: VfState = field(default_factory=VfState)
    DPDKMode: bool = False
    Master: str = ""
    MAC: str = ""
    vlan: int | None = None
    vlanQoS: int | None = None
    vlanProto: str | None = None
    deviceID: str = ""
    VFID: int = 0
    min_tx_rate: int | None = None
    max_tx_rate: int | None = None
    spoofchk: str = ""
    trust: str = ""
    link_state: str = ""
    runtimeConfig: dict = field(default_factory=dict)
    logLevel: str = ""
    logFile: str = ""
    raw: dict = field(default_factory=dict)

    def to_json(self) -> dict:
        d = dict(self.raw)
        for k in ("cniVersion", "name", "type", "MAC", "deviceID", "VFID", "Master", "DPDKMode"):
            d[k] = getattr(self, k)
        for k in ("vlan", "vlanQoS", "vlanProto", "min_tx_rate", "max_tx_rate"):
            if getattr(self, k) is not None:
                d[k] = getattr(self, k)
        for k in ("spoofchk", "trust", "link_state", "logLevel", "logFile"):
            if getattr(self, k):
                d[k] = getattr(self, k)
        if self.ipam:
            d["ipam"] = self.ipam
        d["OrigVfState"] = self.OrigVfState.__dict__
        return d


@dataclass
class PodRequest:
    command: str
    pod_namespace: str = ""
    pod_name: str = ""
    pod_uid: str = ""
    container_id: str = ""
    netns: str = ""
    ifname: str = "eth0"
    path: str = ""
    cni_conf: NetConf | None = None
    cni_req: Request | None = None
    timestamp: float = field(default_factory=time.time)
    deadline: float = field(default_factory=lambda: time.time() + 120.0)  # 2 min (cniserver.go)
    net_name: str = ""
    device_info: dict = field(default_factory=dict)
    cancelled: threading.Event = field(default_factory=threading.Event)

    def env(self) -> dict[str, str]:
        return {"CNI_COMMAND": self.command, "CNI_CONTAINERID": self.container_id, "CNI_NETNS": self.netns,
                "CNI_IFNAME": self.ifname, "CNI_PATH": self.path}


def result_json(version: str, interfaces=None, ips=None, routes=None, dns=None) -> dict:
    """A CNI Result (types/100 layout)."""
    return {"cniVersion": version, "interfaces": interfaces or [], "ips": ips or [], "routes": routes or [],
            "dns": dns or {}}
