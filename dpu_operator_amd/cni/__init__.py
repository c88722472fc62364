"""dpu-cni: CNI shim, unix-socket CNI server, NF/SR-IOV attach (reference: dpu-cni/)."""
