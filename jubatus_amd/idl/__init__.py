"""jubatus_amd.idl"""
