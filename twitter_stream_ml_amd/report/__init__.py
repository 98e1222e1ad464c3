"""report"""
