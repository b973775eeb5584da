# MI355X node image: PyTorch-ROCm base, in-tree gfx950 kernels and the
# native RESP server built at image build time.  Run with the GPUs and the
# KFD device mapped in, e.g.
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video \
#     --ipc=host -e RESOURCE_NAME=worker -e REDIS_HOST=redis-master <image>
ARG BASE=rocm/pytorch:latest
FROM ${BASE}

ENV PYTHONUNBUFFERED=1 \
    PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0

WORKDIR /opt/kiosk-autoscaler

COPY requirements.txt .
RUN pip install --no-cache-dir -r requirements.txt

COPY . .
# hipcc --offload-arch=gfx950 (cross-compiles; no GPU needed at build time)
RUN python tools/build_native.py

# the reference's entry point: reconcile loop configured by env variables
CMD ["python", "scale.py"]
