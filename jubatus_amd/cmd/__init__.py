"""jubatus_amd.cmd"""
