"""Exception hierarchy (reference: veles/error.py:38-60)."""


class VelesException(Exception):
    pass


class BadFormatError(VelesException):
    pass


class AlreadyExistsError(VelesException):
    pass


class NotExistsError(VelesException):
    pass


class MasterSlaveCommunicationError(VelesException):
    pass


class DeviceNotFoundError(VelesException):
    pass


class Bug(VelesException):
    pass


class KernelLibraryMissing(VelesException):
    """Raised when a GPU op is requested but the HIP kernel library is absent."""
