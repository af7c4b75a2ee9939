"""Model file container (reference C21: jubatus/server/framework/save_load.cpp).

Layout (all integers big-endian)::

    [0:8)    "jubatus\\0"                      magic
    [8:16)   format version (u64) = 1
    [16:28)  jubatus major, minor, maintenance (u32 x3)
    [28:32)  CRC32 of header[0:28] ++ header[32:48] ++ system ++ user
    [32:40)  system_data size (u64)
    [40:48)  user_data size (u64)
    system_data = msgpack [version=1, timestamp, type, id, config]
    user_data   = msgpack [user_data_version, <driver pack>]

Load checks magic, format version, exact jubatus version, CRC, system data
version, server type and (unless the file's config is adopted) semantic
config equality (JSON-normalised compare), then the user data version.
``<driver pack>`` is our own documented payload: each driver's
``pack()`` object (see jubatus_amd/models/*).
"""
from __future__ import annotations

import json
import struct
import time
from typing import Any, BinaryIO

import msgpack

from .. import JUBATUS_VERSION
from .._native import native
from ..common.mprpc import packb, unpackb

MAGIC = b"jubatus\x00"
FORMAT_VERSION = 1
SYSTEM_DATA_VERSION = 1
HEADER = struct.Struct(">8sQIIIIQQ")  # 48 bytes


class ModelFileError(ValueError):
    pass


def _crc(header: bytes, system: bytes, user: bytes) -> int:
    n = native()
    c = n.crc32(header[0:28])
    c = n.crc32(header[32:48], c)
    c = n.crc32(system, c)
    return n.crc32(user, c)


def compare_config(a: str, b: str) -> bool:
    try:
        return json.dumps(json.loads(a), sort_keys=True) == json.dumps(json.loads(b), sort_keys=True)
    except (json.JSONDecodeError, TypeError):
        return a == b


def save_server(fp: BinaryIO, server_type: str, model_id: str, config: str,
                user_data_version: int, driver_pack: Any) -> None:
    system = packb([SYSTEM_DATA_VERSION, int(time.time()), server_type, model_id, config])
    # user data: bin type so model blobs round-trip as bytes (our own payload;
    # the system data keeps the reference's old-spec RAW strings)
    user = msgpack.packb([int(user_data_version), driver_pack], use_bin_type=True)
    major, minor, maint = JUBATUS_VERSION
    head = bytearray(HEADER.pack(MAGIC, FORMAT_VERSION, major, minor, maint, 0, len(system),
                                 len(user)))
    struct.pack_into(">I", head, 28, _crc(bytes(head), system, user))
    fp.write(bytes(head))
    fp.write(system)
    fp.write(user)


def read_model_file(fp: BinaryIO) -> tuple[list, list]:
    """Validated (system_data, user_data) of a model file; raises ModelFileError."""
    head = fp.read(48)
    if len(head) != 48:
        raise ModelFileError("failed to read header: truncated file")
    magic, fmt, major, minor, maint, crc, ssz, usz = HEADER.unpack(head)
    if magic != MAGIC:
        raise ModelFileError("invalid file format")
    if fmt != FORMAT_VERSION:
        raise ModelFileError(f"invalid format version: {fmt}, expected {FORMAT_VERSION}")
    if (major, minor, maint) != tuple(JUBATUS_VERSION):
        raise ModelFileError(f"jubatus version mismatched: current version: "
                             f"{'.'.join(map(str, JUBATUS_VERSION))}, saved version: "
                             f"{major}.{minor}.{maint}")
    system = fp.read(ssz)
    user = fp.read(usz)
    if len(system) != ssz or len(user) != usz:
        raise ModelFileError("model file truncated")
    actual = _crc(head, system, user)
    if actual != crc:
        raise ModelFileError(f"invalid crc32 checksum: {actual:#x}, read {crc:#x}")
    try:
        sysobj = unpackb(system)
        userobj = unpackb(user)
    except Exception as e:
        raise ModelFileError(f"broken model data: {e}") from e
    if not isinstance(sysobj, list) or len(sysobj) != 5:
        raise ModelFileError("invalid system data")
    if not isinstance(userobj, list) or len(userobj) != 2:
        raise ModelFileError("invalid user data")
    return sysobj, userobj


def load_server(fp: BinaryIO, server_type: str, current_config: str | None,
                user_data_version: int, overwrite_config: bool) -> tuple[str, Any]:
    """-> (config string to use, driver pack object)."""
    sysobj, userobj = read_model_file(fp)
    version, _ts, typ, _id, config = sysobj
    if version != SYSTEM_DATA_VERSION:
        raise ModelFileError(f"invalid system data version: saved version: {version}, "
                             f"expected version: {SYSTEM_DATA_VERSION}")
    if typ != server_type:
        raise ModelFileError(f"invalid model type: saved type: {typ}, expected type: {server_type}")
    if not overwrite_config and current_config is not None and not compare_config(config, current_config):
        raise ModelFileError("model config mismatched with the running config")
    if userobj[0] != user_data_version:
        raise ModelFileError(f"user data version mismatched: {userobj[0]}, current version: "
                             f"{user_data_version}")
    return config, userobj[1]
