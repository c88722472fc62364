"""Shared constants (reference: pkgs/vars/vars.go:3-13)."""

NAMESPACE = "openshift-dpu-operator"
DPU_OPERATOR_CONFIG_NAME = "dpu-operator-config"
DEFAULT_HOST_NAD_NAME = "default-sriov-net"
NF_NAD_NAME = "dpunfcni-conf"
METRICS_SERVICE_NAME = "dpu-operator-controller-manager-metrics-service"
RESOURCE_NAME = "openshift.io/dpu"          # extended resource advertised by the device plugin
NRI_CONTROL_SWITCH_CM = "nri-control-switches"
