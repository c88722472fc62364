from .environment import ClusterEnvironment, FilesystemModeDetector  # noqa: F401
from .paths import FilesystemMode, Flavour, PathManager  # noqa: F401
