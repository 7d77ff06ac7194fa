"""Input pipeline: TFRecord loader (C++), sharding policies, synthetic Criteo-shape data."""
