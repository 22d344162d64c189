# Container image (reference: Dockerfile:1-6 - FROM tritonmedia/base, yarn install, uid 999).
# ROCm userspace is needed only for the optional gfx950 piece-verification module; the
# staging path itself is host-side (native C++ + asyncio).
FROM rocm/dev-ubuntu-22.04:7.2

RUN apt-get update && apt-get install -y --no-install-recommends \
        python3 python3-pip python3-dev g++ libssl-dev && \
    rm -rf /var/lib/apt/lists/*

WORKDIR /app
COPY pyproject.toml README.md ./
RUN pip3 install --no-cache-dir aiohttp protobuf pydantic pyyaml prometheus_client pybind11 numpy

COPY downloader_amd ./downloader_amd
COPY __graft_entry__.py bench.py ./
RUN PYTORCH_ROCM_ARCH=gfx950 python3 -m downloader_amd.ops.build

RUN useradd -u 999 -m stager && mkdir -p /app/downloads && chown -R 999:999 /app
USER 999
ENV PORT=3401 LOG_LEVEL=info
EXPOSE 3401
HEALTHCHECK --interval=30s --timeout=5s CMD python3 -c "import urllib.request,sys; urllib.request.urlopen('http://127.0.0.1:3401/healthz', timeout=3)" || exit 1
CMD ["python3", "-m", "downloader_amd", "worker"]
