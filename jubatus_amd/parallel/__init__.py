"""jubatus_amd.parallel"""
