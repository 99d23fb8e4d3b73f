"""Distributed execution: process groups, partition ownership, collectives."""
