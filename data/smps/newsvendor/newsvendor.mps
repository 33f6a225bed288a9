* ENCODING=ISO-8859-1
NAME          
ROWS
 N  obj1    
 G  con1    
 G  con2    
 E  con3    
COLUMNS
    x         con1                           -1
    x         con2                            1
    y1        obj1                          0.5
    y1        con1                            1
    y2        obj1                            4
    y2        con2                            1
    y3        con1                            1
    y3        con2                           -1
    y3        con3                            1
RHS
    rhs       con3                            5
BOUNDS
 UP bnd       x                              10
ENDATA
