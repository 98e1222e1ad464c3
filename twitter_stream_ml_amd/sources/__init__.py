"""sources"""
