from .v1 import (  # noqa: F401
    API_VERSION,
    KIND_DPU_OPERATOR_CONFIG,
    KIND_SFC,
    DpuOperatorConfig,
    DpuOperatorConfigSpec,
    NetworkFunction,
    ServiceFunctionChain,
    ValidationError,
    crd_manifests,
    validate_dpu_operator_config,
    validate_sfc,
)
