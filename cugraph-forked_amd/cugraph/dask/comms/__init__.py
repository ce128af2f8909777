from . import comms  # noqa: F401
