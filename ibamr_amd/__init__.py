"""MI355X-native LE coupling path of IBAMR (IBTK LEInteractor::spread / interpolate)."""
