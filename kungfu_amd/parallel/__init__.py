"""Device data plane (RCCL) and the bucketed gradient engine."""
from .comm import DeviceComm, destroy_device_comm, get_device_comm, reset_device_comm
from .flat import FlatParamSpace
