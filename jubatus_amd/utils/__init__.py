"""jubatus_amd.utils"""
