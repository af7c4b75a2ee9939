"""jubatus_amd.framework"""
