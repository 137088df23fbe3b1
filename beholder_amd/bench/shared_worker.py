"""``python -m beholder_amd.bench.shared_worker run ...``: the service's own ``run`` command
(beholder_amd.cli), with one change for the shared-queue bench (bench/shared_queue.py): every
sink request is answered by the in-process stub of the headline (sinks/http.py
RecordingHttpClient, h1 stub: the H1 client's request bytes and response parsing, no socket)
instead of going to Trello / Telegram / Emby. With ``--workers N`` the supervisor starts this
module for each worker (it names itself in ``BEHOLDER_WORKER_MODULE``, cli.worker_command), so every
worker has the stub too.
"""
from __future__ import annotations

import os
import sys


def main(argv=None) -> int:
    from .. import service
    from ..cli import WORKER_MODULE_ENV
    os.environ[WORKER_MODULE_ENV] = "beholder_amd.bench.shared_worker"  # every worker runs this module too
    from ..sinks import RecordingHttpClient

    def stub_client(http_cfg):
        return RecordingHttpClient(keep=0)
    service.make_http_client = stub_client
    from ..cli import main as cli_main
    return cli_main(sys.argv[1:] if argv is None else argv)


if __name__ == "__main__":
    raise SystemExit(main())
