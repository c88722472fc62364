"""CNI-aware logging: every line carries cniName / containerID / netns / ifname.

Reference: dpu-cni/pkgs/cnilogging/cnilogging.go:26-93 (a cni-log wrapper prepending those labels;
log level / file taken from the NetConf).
"""
from __future__ import annotations

import logging
import sys

_LEVELS = {"panic": logging.CRITICAL, "error": logging.ERROR, "warning": logging.WARNING,
           "info": logging.INFO, "debug": logging.DEBUG, "verbose": logging.DEBUG}
_state = {"name": "", "cid": "", "netns": "", "ifname": ""}
_logger = logging.getLogger("dpu-cni")


def init(log_level: str = "info", log_file: str = "", stderr=None) -> None:
    _logger.handlers.clear()
    h = logging.FileHandler(log_file) if log_file else logging.StreamHandler(stderr or sys.stderr)
    h.setFormatter(logging.Formatter("%(asctime)s [%(levelname)s] %(message)s"))
    _logger.addHandler(h)
    _logger.setLevel(_LEVELS.get((log_level or "info").lower(), logging.INFO))
    _logger.propagate = False


def set_labels(cni_name: str = "", container_id: str = "", netns: str = "", ifname: str = "") -> None:
    _state.update(name=cni_name, cid=container_id, netns=netns, ifname=ifname)


def _prefix(msg: str, kv: dict) -> str:
    parts = [f'cniName="{_state["name"]}"', f'containerID="{_state["cid"]}"', f'netns="{_state["netns"]}"',
             f'ifname="{_state["ifname"]}"']
    parts += [f'{k}="{v}"' for k, v in kv.items()]
    return f"{msg} " + " ".join(parts)


def debug(msg: str, **kv) -> None:
    _logger.debug(_prefix(msg, kv))


def info(msg: str, **kv) -> None:
    _logger.info(_prefix(msg, kv))


def warning(msg: str, **kv) -> None:
    _logger.warning(_prefix(msg, kv))


def error(msg: str, **kv) -> None:
    _logger.error(_prefix(msg, kv))
