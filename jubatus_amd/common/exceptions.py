"""Exception taxonomy shared by servers and clients (reference
jubatus/server/common/mprpc/exception.hpp and jubatus_core's
jubatus_exception family)."""


class ArgumentError(TypeError):
    """Bad RPC argument (arity / type); the RPC layer answers ARGUMENT_ERROR."""


class ConfigNotSet(RuntimeError):
    def __init__(self):
        super().__init__("config_not_set")


class UnsupportedMethod(RuntimeError):
    pass
