"""pysignalduino_amd — MI355X-native batched SIGNALduino MU/MS/MC demodulator.

Drop-in for the ``sd_protocols.SDProtocols`` demodulation path of
RFD-FHEM/PySignalduino.  The compute path is hand-written HIP
for gfx950 behind the C-ABI declared in ``include/sdx.h``.
"""
__version__ = "0.1.0"
