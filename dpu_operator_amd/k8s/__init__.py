"""In-process Kubernetes emulation used by the control plane (see apiserver.py)."""
from .apiserver import (  # noqa: F401
    AlreadyExists,
    ApiError,
    ApiServer,
    BadRequest,
    Conflict,
    Forbidden,
    NotFound,
    is_not_found,
    make_node,
    owner_reference,
    set_controller_reference,
)
from .manager import Manager, Request, Result  # noqa: F401
