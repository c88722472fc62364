from .operator import (  # noqa: F401
    DpuOperatorConfigReconciler,
    ServiceFunctionChainReconciler,
    install_webhook,
    setup_operator,
)
