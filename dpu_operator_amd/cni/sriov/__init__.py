"""Host-side SR-IOV VF attach (sriov-cni equivalent)."""
from .manager import SriovManager, SriovManagerStub, load_conf  # noqa: F401
from .pci_allocator import PCIAllocator  # noqa: F401
from .utils import Sysfs, is_valid_pci_address  # noqa: F401
