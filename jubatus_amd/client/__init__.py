"""jubatus_amd.client"""
