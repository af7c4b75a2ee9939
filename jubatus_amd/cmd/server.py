"""juba<engine> entry point: ``python -m jubatus_amd.cmd.server <engine> [flags]``
(bin/juba<engine> wraps this). Same flags as the reference servers."""
from __future__ import annotations

import sys


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    from ..server import SERVERS, get_serv
    if not argv or argv[0] not in SERVERS:
        sys.stderr.write(f"usage: server <{'|'.join(SERVERS)}> [options]\n")
        return 1
    engine = argv.pop(0)
    from ..framework.server_helper import run_server
    return run_server(get_serv(engine), argv, engine, prog=f"juba{engine}")


if __name__ == "__main__":
    sys.exit(main())
