from .registry import (  # noqa: F401
    DEVICE_PLUGIN_VERSION,
    HEALTHY,
    UNHEALTHY,
    GoogleEmpty,
    deviceplugin,
    opi,
    p4rt,
    vendor,
)
