# Container images of the framework (reference: Dockerfile.rhel, Dockerfile.daemon.rhel,
# Dockerfile.*VSP.rhel, Dockerfile.networkResourcesInjector.rhel, Dockerfile.mrvlCPAgent.rhel).
# One multi-stage file: `docker build --target <operator|daemon|vsp-gpu|nri|p4rt-server|cp-agent> .`
#
# BASE must provide ROCm 7.x + PyTorch (ROCm build) + Python 3.10 — the same stack the data plane
# is built and tested on.  The HIP extension is compiled for gfx950 (MI355X) only.
ARG BASE=rocm/pytorch:latest

FROM ${BASE} AS build
WORKDIR /src
COPY csrc csrc
COPY dpu_operator_amd dpu_operator_amd
COPY __graft_entry__.py .
RUN python3 -m pip install --no-cache-dir pybind11 grpcio protobuf pyyaml && \
    PYTORCH_ROCM_ARCH=gfx950 python3 -m dpu_operator_amd.native.build -v

FROM ${BASE} AS runtime
RUN python3 -m pip install --no-cache-dir grpcio protobuf pyyaml
WORKDIR /opt/dpu-operator
COPY --from=build /src/dpu_operator_amd dpu_operator_amd
ENV PYTHONPATH=/opt/dpu-operator

# cluster operator (O1): reconciles DpuOperatorConfig / ServiceFunctionChain
FROM runtime AS operator
USER 65532:65532
ENTRYPOINT ["python3", "-m", "dpu_operator_amd.cmd.operator"]

# node daemon (N2): the static dpu-cni binary is installed onto the host from /dpu-cni
FROM runtime AS daemon
COPY --from=build /src/dpu_operator_amd/native/bin/dpu-cni /dpu-cni
ENTRYPOINT ["python3", "-m", "dpu_operator_amd.cmd.daemon"]

# vendor plugin on the MI355X data plane (GPU VSP); also serves mock / marvell / netsec / intel
FROM runtime AS vsp-gpu
ENTRYPOINT ["python3", "-m", "dpu_operator_amd.cmd.vsp", "--vendor", "amd-gpu"]

# network resources injector (N1)
FROM runtime AS nri
USER 65532:65532
ENTRYPOINT ["python3", "-m", "dpu_operator_amd.cmd.nri"]

# P4Runtime pipeline server (V13 role)
FROM runtime AS p4rt-server
ENTRYPOINT ["python3", "-m", "dpu_operator_amd.cmd.p4rt_server"]

# native control-plane agent (NAT1): no Python needed
FROM ${BASE} AS cp-agent
COPY --from=build /src/dpu_operator_amd/native/bin/dpu-cp-agent /usr/local/bin/dpu-cp-agent
ENTRYPOINT ["/usr/local/bin/dpu-cp-agent"]
