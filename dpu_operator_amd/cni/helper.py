"""CNI request helpers (reference: dpu-cni/pkgs/cnihelper/cnihelper.go:15-52)."""
from __future__ import annotations

import json
import os

from .types import NetConf, Request, VfState

_NETCONF_FIELDS = set(NetConf.__dataclass_fields__) - {"raw", "OrigVfState"}


def new_cni_request(env: dict | None = None, stdin: bytes = b"") -> Request:
    """Snapshot the CNI_* environment + stdin config into a Request (what the shim sends)."""
    env = dict(os.environ if env is None else env)
    keep = {k: v for k, v in env.items() if k.startswith("CNI_")}
    return Request(env=keep, config=stdin)


def _go_fields(d: dict, fields: set[str]) -> dict:
    """Map JSON keys onto field names the way Go's encoding/json does: an exact key wins, else a
    case-insensitive match (so `"EffectiveMac"` fills EffectiveMAC, as the reference's tests use)."""
    lower = {f.lower(): f for f in fields}
    out: dict = {}
    for k, v in d.items():
        if k in fields:
            out[k] = v
        elif k.lower() in lower and lower[k.lower()] not in d:
            out.setdefault(lower[k.lower()], v)
    return out


def read_cni_config(b: bytes) -> NetConf:
    """Parse a network config (JSON) including an optional prevResult."""
    try:
        d = json.loads(b.decode() if isinstance(b, (bytes, bytearray)) else b)
    except (ValueError, UnicodeDecodeError) as e:
        raise ValueError(f"failed to parse network config: {e}") from e
    if not isinstance(d, dict):
        raise ValueError("network config must be a JSON object")
    conf = NetConf(raw=d)
    for k, v in _go_fields(d, _NETCONF_FIELDS).items():
        setattr(conf, k, v)
    ovs = _go_fields(d, {"OrigVfState"}).get("OrigVfState")
    if isinstance(ovs, dict):
        conf.OrigVfState = VfState(**_go_fields(ovs, set(VfState.__dataclass_fields__)))
    if conf.prevResult is not None and not isinstance(conf.prevResult, dict):
        raise ValueError("prevResult must be an object")
    return conf
