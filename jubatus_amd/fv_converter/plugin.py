"""fv_converter plug-in loader (``"method": "dynamic"``).

Placeholder until the native plug-in ABI lands; see
jubatus/server/fv_converter/dynamic_loader.cpp:44-94 for the reference
search order ($JUBATUS_PLUGIN_PATH, then the install plugin dir).
"""
from __future__ import annotations


class PluginError(RuntimeError):
    pass


class PluginLoader:
    def create(self, kind: str, params: dict):
        raise PluginError(f"dynamic {kind} plugins are not available yet")
