"""juba<engine>_proxy entry point: ``python -m jubatus_amd.cmd.proxy <engine> [flags]``."""
from __future__ import annotations

import sys


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    from ..idl import specs
    if not argv or argv[0] not in specs.SERVICES:
        sys.stderr.write(f"usage: proxy <{'|'.join(specs.SERVICES)}> [options]\n")
        return 1
    engine = argv.pop(0)
    from ..framework.proxy import run_proxy
    return run_proxy(argv, engine)


if __name__ == "__main__":
    sys.exit(main())
