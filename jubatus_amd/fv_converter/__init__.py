"""jubatus_amd.fv_converter"""
