"""MI355X-native structured-light reconstruction (Gray-code decode + ray-plane triangulation).

Drop-in for the hot path of TtT609/Structured_Light_for_3D_Model_Replication
(``server/processing.py:27-334``, ``server/sl_system.py:491-702``); see DESIGN.md.
"""
__version__ = "0.1.0"
