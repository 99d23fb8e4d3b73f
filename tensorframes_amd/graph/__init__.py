"""Graph layer: GraphDef codec (proto.py) and the TF-1.x-compatible builder (dsl.py)."""
