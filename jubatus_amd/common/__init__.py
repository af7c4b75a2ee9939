"""jubatus_amd.common"""
