"""Strict template rendering + apply of bindata manifests.

Reference: pkgs/render/render.go:25-110 — Go text/template with ``missingkey=error``, one YAML
object per file, files applied in sorted order, controller owner reference to the
DpuOperatorConfig, AlreadyExists / Conflict swallowed.  The template language supported here is
the subset the manifests use: ``{{.Key}}`` / ``{{ .Key }}`` substitution (missing key = error),
plus ``{{- ...}}`` / ``{{... -}}`` whitespace trimming.
"""
from __future__ import annotations

import logging
import re
from importlib import resources
from pathlib import Path

import yaml

from .k8s.apiserver import AlreadyExists, ApiServer, Conflict, set_controller_reference

log = logging.getLogger("dpu.render")

_TOKEN = re.compile(r"(\s*)\{\{(-?)\s*\.([A-Za-z_][A-Za-z0-9_]*)\s*(-?)\}\}(\s*)")


class TemplateError(KeyError):
    pass


def apply_template(text: str, data: dict) -> str:
    def sub(m: re.Match) -> str:
        lead, ltrim, key, rtrim, trail = m.groups()
        if key not in data:
            raise TemplateError(f'map has no entry for key "{key}"')
        return ("" if ltrim else lead) + str(data[key]) + ("" if rtrim else trail)

    out = _TOKEN.sub(sub, text)
    if "{{" in out:
        raise TemplateError(f"unsupported template construct near: {out[out.index('{{'):][:40]!r}")
    return out


def bindata_root() -> Path:
    return Path(str(resources.files("dpu_operator_amd"))) / "bindata"


def bindata_files(subdir: str) -> list[Path]:
    d = bindata_root() / subdir
    if not d.is_dir():
        raise FileNotFoundError(f"no bindata directory {subdir}")
    return sorted(p for p in d.iterdir() if p.is_file() and p.suffix == ".yaml")


def render_file(path: Path, data: dict) -> dict:
    return yaml.safe_load(apply_template(path.read_text(), data))


def apply_all_from_bindata(api: ApiServer, subdir: str, data: dict, owner: dict | None = None) -> list[dict]:
    applied = []
    for f in bindata_files(subdir):
        obj = render_file(f, data)
        if owner is not None:
            set_controller_reference(owner, obj)
        try:
            applied.append(api.apply(obj))
        except AlreadyExists:
            log.info("resource already exists, skipping %s %s", obj.get("kind"), obj["metadata"].get("name"))
        except Conflict:
            log.info("resource conflict, skipping %s %s", obj.get("kind"), obj["metadata"].get("name"))
    return applied
