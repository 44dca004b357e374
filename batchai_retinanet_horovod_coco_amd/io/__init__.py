"""I/O: HDF5 subset (Keras checkpoint layout), checkpoints (h5 / safetensors), TensorBoard events."""
