# Reference: FROM tritonmedia/base; yarn; copy source into /stack as uid 999 (Dockerfile:1-6).
# Two stages: the native runtime is compiled in `build` (g++, OpenSSL headers); the `runtime`
# image gets the package with the built extension and no compiler or headers, and never
# rebuilds on import (BEHOLDER_ALLOW_BUILD=0).

FROM python:3.10-slim AS build
RUN apt-get update && apt-get install -y --no-install-recommends g++ libssl-dev && rm -rf /var/lib/apt/lists/*
WORKDIR /stack
RUN pip install --no-cache-dir --prefix=/install protobuf pyyaml
COPY . /stack
# native runtime (ingest ring, codec, deliveries, metrics, text, TLS) built in-tree; the optional
# gfx950 HIP probe library and the bench/test natives (_native_bench: sink stub, paced producer,
# calibrations, profiler) are not built: the image ships only the service
RUN python -m beholder_amd._build --force --no-hip --no-bench \
    && rm -rf beholder_amd/ops/csrc beholder_amd/ops/csrc_bench beholder_amd/ops/*.lock tests profiles scripts \
    && find /stack -name __pycache__ -prune -exec rm -rf {} +

FROM python:3.10-slim AS runtime
WORKDIR /stack
RUN useradd --uid 999 --create-home --home-dir /home/beholder beholder && chown 999:999 /stack
COPY --from=build /install /usr/local
COPY --from=build --chown=999:999 /stack /stack
USER 999
ENV CONFIG_PATH=/stack/config \
    BEHOLDER_ALLOW_BUILD=0
EXPOSE 3000
ENTRYPOINT ["python", "-m", "beholder_amd", "run"]
