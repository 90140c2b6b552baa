"""emqx_amd -- MI355X-native topic matching for EMQX's publish-routing hot path.

Host mirror of the reference interfaces (``topic_index``, ``router``) over the
C ABI of ``libtmatch.so`` (``include/tmatch.h``): a device-resident index of
MQTT topic filters matched by hand-written gfx950 kernels.
"""
__version__ = "0.1.0"
