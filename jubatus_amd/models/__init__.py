"""jubatus_amd.models"""
