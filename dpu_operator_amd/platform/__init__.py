from .detectors import (  # noqa: F401
    DpuDetectorManager,
    IntelIpuDetector,
    MarvellDetector,
    Mi355xDetector,
    NetsecAcceleratorDetector,
    VspSpec,
)
from .platform import FakePlatform, Nic, PciDevice, Platform, SysfsPlatform  # noqa: F401
