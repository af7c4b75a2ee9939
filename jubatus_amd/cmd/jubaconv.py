"""jubaconv: offline fv_converter debugger (reference C34,
jubatus/server/cmd/jubaconv.cpp:47-198).

stdin JSON -> datum -> feature vector. ``-i json|datum``, ``-o
json|datum|fv``, ``-c server_config.json`` (its ``converter`` section).
JSON -> datum flattening (core json_converter, EXTERNAL; parity unpinned):
object keys join as "/a/b", array elements as "/a[0]", strings go to
string_values, numbers to num_values, booleans to num_values as 1/0, nulls
are skipped. A datum on stdin is {"string_values": [[k, v]...],
"num_values": [[k, x]...], "binary_values": [[k, b]...]}. fv lines are
"<feature>: <value>".
"""
from __future__ import annotations

import argparse
import json
import sys

from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum


def json_to_datum(obj, prefix: str = "", d: Datum | None = None) -> Datum:
    d = d if d is not None else Datum()
    if isinstance(obj, dict):
        for k, v in obj.items():
            json_to_datum(v, f"{prefix}/{k}", d)
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            json_to_datum(v, f"{prefix}[{i}]", d)
    elif isinstance(obj, bool):
        d.num_values.append((prefix, 1.0 if obj else 0.0))
    elif isinstance(obj, (int, float)):
        d.num_values.append((prefix, float(obj)))
    elif isinstance(obj, str):
        d.string_values.append((prefix, obj))
    return d


def datum_to_json(d: Datum) -> dict:
    return {"string_values": [list(x) for x in d.string_values],
            "num_values": [list(x) for x in d.num_values],
            "binary_values": [[k, v.decode("latin-1") if isinstance(v, bytes) else v]
                              for k, v in d.binary_values]}


def datum_from_json(obj: dict) -> Datum:
    d = Datum()
    d.string_values = [(str(k), str(v)) for k, v in obj.get("string_values", [])]
    d.num_values = [(str(k), float(v)) for k, v in obj.get("num_values", [])]
    d.binary_values = [(str(k), v.encode("latin-1") if isinstance(v, str) else bytes(v))
                       for k, v in obj.get("binary_values", [])]
    return d


def main(argv: list[str] | None = None, stdin=None, out=None) -> int:
    stdin = stdin or sys.stdin
    out = out or sys.stdout
    p = argparse.ArgumentParser(prog="jubaconv")
    p.add_argument("-i", "--input-format", default="json", choices=("json", "datum"))
    p.add_argument("-o", "--output-format", default="fv", choices=("json", "datum", "fv"))
    p.add_argument("-c", "--conf", default="")
    a = p.parse_args(argv)
    try:
        data = json.load(stdin)
    except json.JSONDecodeError:
        sys.stderr.write(f"invalid {a.input_format} format\n")
        return -1
    if a.output_format == "json":
        if a.input_format != "json":
            sys.stderr.write(f"invalid input-output type: {a.input_format} -> json\n")
            return -1
        out.write(json.dumps(data, indent=2) + "\n")
        return 0
    d = datum_from_json(data) if a.input_format == "datum" else json_to_datum(data)
    if a.output_format == "datum":
        out.write(json.dumps(datum_to_json(d), indent=2) + "\n")
        return 0
    if not a.conf:
        sys.stderr.write("specify converter config with -c flag\n")
        return -1
    try:
        with open(a.conf) as f:
            conf = json.load(f)
    except OSError:
        sys.stderr.write(f"cannot open converter config file: {a.conf}\n")
        return -1
    conv = DatumToFvConverter(conf.get("converter") or {})
    for name, v in conv.convert(d):
        out.write(f"{name}: {v:g}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
