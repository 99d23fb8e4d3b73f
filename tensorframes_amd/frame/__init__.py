"""DataFrame substrate: schema types, tensor metadata, columnar partitions."""
