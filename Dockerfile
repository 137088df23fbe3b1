# Reference: FROM tritonmedia/base; yarn; copy source into /stack as uid 999 (Dockerfile:1-6).
FROM python:3.10-slim

RUN apt-get update && apt-get install -y --no-install-recommends g++ libssl-dev && rm -rf /var/lib/apt/lists/*
WORKDIR /stack
RUN useradd --uid 999 --create-home --home-dir /home/beholder beholder && chown 999:999 /stack

COPY --chown=999:999 pyproject.toml /stack/
RUN pip install --no-cache-dir protobuf pyyaml
COPY --chown=999:999 . /stack
# native runtime (ingest ring, codec, deliveries, metrics, text) built in-tree; the optional gfx950
# HIP probe library is skipped here (no hipcc in this image)
RUN python -m beholder_amd.ops.build --force && chown -R 999:999 /stack

USER 999
ENV CONFIG_PATH=/stack/config
EXPOSE 3000
ENTRYPOINT ["python", "-m", "beholder_amd", "run"]
