"""jubatus_amd.server"""
