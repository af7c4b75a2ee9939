"""jubatus_amd.ops"""
