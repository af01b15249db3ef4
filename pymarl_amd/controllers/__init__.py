REGISTRY = {}

from .basic_controller import BasicMAC  # noqa: E402

REGISTRY["basic_mac"] = BasicMAC
