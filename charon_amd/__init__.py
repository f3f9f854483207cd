"""charon_amd: MI355X-native BLS12-381 engine for charon's tbls hot path."""
