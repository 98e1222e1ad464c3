"""checkpoint"""
